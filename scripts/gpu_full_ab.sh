# Whole -m gpu suite on the product build, then A/B of named builds (scripts/ab_probe.py).
# Usage: bash scripts/gpu_full_ab.sh "libA libB ..." "--c2 ..."
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/full_tests.log
[ $rc -eq 0 ] || exit 1
L=""; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 500 python -u scripts/ab_probe.py $L $2 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
