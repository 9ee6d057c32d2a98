# Quick GPU check: smoke, the -m gpu suite, a C2 bench line.
# Usage: bash scripts/gpu_check.sh [pytest -k expression]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail gpurun_out/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print(d['value'], d['ms_per_step'], d['wall_ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
