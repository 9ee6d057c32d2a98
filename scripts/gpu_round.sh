# Closing-style run on the GPU box: the whole -m gpu suite, smoke(), and the driver's default bench
# line (gpurun_out/TAG_bench.json; full records in gpurun_out/TAG_bench_full.json).
# Usage: bash scripts/gpu_round.sh TAG [pytest -k expression]
TAG=${1:-r6}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
K=${2:+-k "$2"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 600 python bench.py --full-json gpurun_out/${TAG}_bench_full.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
wc -c gpurun_out/${TAG}_bench.json
python scripts/bench_summary.py gpurun_out/${TAG}_bench.json 2>/dev/null || cat gpurun_out/${TAG}_bench.json
