# GPU session for kernel A/B work: quick parity suite on the default build, then interleaved A/B of
# every raft-simulation_amd/build/libraftsim*.so in one process (scripts/ab_probe.py).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_fuzz.py tests/test_golden.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/quick_tests.log
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python -u scripts/ab_probe.py raft-simulation_amd/build/libraftsim*.so > gpurun_out/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab.log
  timeout -k 10 120 python -u scripts/occ_probe.py > gpurun_out/occ.log 2>&1; echo "occ rc=$?"; cat gpurun_out/occ.log
fi
