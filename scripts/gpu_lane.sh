# Steady-path parity tests and an A/B of the default build against variants (one call).
# Usage: bash scripts/gpu_lane.sh "variant-libs" "ab-args" ["pytest -k expr"]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
K=${3:-"steady or lite or c2"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/lane_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/lane_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert|differ" gpurun_out/lane_tests.log | head -30; exit 1; }
L="$B/libraftsim.so"; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 300 python -u scripts/ab_probe.py $L $2 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
