# Quick GPU iteration: parity subset + throughput probe.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_fuzz.py tests/test_golden.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/quick_tests.log
if [ $rc -eq 0 ]; then timeout -k 10 300 python scripts/perf_probe.py > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe.log; fi
