cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
L=raft-simulation_amd/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_windows.py -x -v --timeout 200 --timeout-method thread -k "steady or lite or c2 or host_writes" > gpurun_out/r5b_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r5b_tests.log | head; tail -30 gpurun_out/r5b_tests.log; exit 1; }
tail -2 gpurun_out/r5b_tests.log
timeout -k 10 120 python scripts/dispatch_probe.py $L/libraftsim_r4.so $L/libraftsim.so > gpurun_out/r5b_probe.txt 2>&1 || { echo "probe failed"; tail gpurun_out/r5b_probe.txt; exit 1; }
cat gpurun_out/r5b_probe.txt
timeout -k 10 120 python scripts/lane_timeline.py $L/libraftsim_wavelog.so > gpurun_out/r5b_timeline.txt 2>&1 || { echo "timeline failed"; tail gpurun_out/r5b_timeline.txt; exit 1; }
cat gpurun_out/r5b_timeline.txt
