# Round-5 working session on the GPU box: the -m gpu suite (or a -k subset), the C2 dispatch A/B
# against the libraries given, and the C2 lane timeline of the -DRS_WAVELOG build.
# Usage: bash scripts/r5_session.sh "[pytest -k expression, empty for all]" [LIB ...]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
L=raft-simulation_amd/build
KEXPR=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/r5_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r5_tests.log | head; tail -30 gpurun_out/r5_tests.log; exit 1; }
tail -2 gpurun_out/r5_tests.log
timeout -k 10 120 python scripts/dispatch_probe.py "$@" $L/libraftsim.so > gpurun_out/r5_probe.txt 2>&1 || { echo "probe failed"; tail gpurun_out/r5_probe.txt; exit 1; }
cat gpurun_out/r5_probe.txt
timeout -k 10 120 python scripts/lane_timeline.py $L/libraftsim_wavelog.so > gpurun_out/r5_timeline.txt 2>&1 || { echo "timeline failed"; tail gpurun_out/r5_timeline.txt; exit 1; }
cat gpurun_out/r5_timeline.txt
