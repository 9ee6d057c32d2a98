# Full -m gpu suite, A/B of builds, then per-wave timelines of a wavelog build (diagnostic).
# Usage: bash scripts/gpu_session2.sh "ab-libs" "ab-args" "wl-libs" "wl-counts"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/full_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/full_tests.log | head -20; exit 1; }
L=""; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 500 python -u scripts/ab_probe.py $L $2 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
[ $rc -eq 0 ] || exit 1
for w in $3; do for c in $4; do
  timeout -k 10 180 python -u scripts/wavelog_probe.py $B/$w.so $c c2 > gpurun_out/wl_${w}_$c.log 2>&1; rc=$?; echo "== wl $w $c rc=$rc"; grep -E "kernel_ms|life|start us|active ticks|started|phase cycles|per-SIMD" gpurun_out/wl_${w}_$c.log
  [ $rc -eq 0 ] || exit 1
done; done
