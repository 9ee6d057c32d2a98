# Quick parity suite on the default build, then A/B of named builds (scripts/ab_probe.py).
# Usage: bash scripts/gpu_ab.sh "libA libB ..." "--c2 --c3 ..."
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_fuzz.py tests/test_golden.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit 1
L=""; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 500 python -u scripts/ab_probe.py $L $2 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
