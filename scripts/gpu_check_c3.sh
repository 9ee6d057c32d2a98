# Targeted parity tests, then the C3-from-init window of named builds (scripts/c3_window.py).
# Usage: bash scripts/gpu_check_c3.sh "pytest -k expr" CLUSTERS STEPS "libs"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$1" --timeout 600 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit 1
L=""; for x in $4; do L="$L $B/$x.so"; done
timeout -k 10 600 python -u scripts/c3_window.py $2 $3 $L > gpurun_out/c3w.log 2>&1; rc=$?; echo "c3w rc=$rc"; cat gpurun_out/c3w.log
