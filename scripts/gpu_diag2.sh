# Diagnostic GPU session (never the product path): per-wave timelines of the RS_WAVELOG builds on
# C2, the occupancy sweep and A/B timing of the product build against named variants.
# Usage: bash scripts/gpu_diag2.sh "wl-libs" "occ-libs" "ab-libs" "ab-args"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
for w in $1; do
  timeout -k 10 180 python -u scripts/wavelog_probe.py $B/$w.so 65536 c2 > gpurun_out/wl_$w.log 2>&1; rc=$?; echo "wl $w rc=$rc"; cat gpurun_out/wl_$w.log
  [ $rc -eq 0 ] || exit 1
done
L=""; for x in $2; do L="$L $B/$x.so"; done
if [ -n "$L" ]; then
  timeout -k 10 300 python -u scripts/occ_probe.py $L > gpurun_out/occ.log 2>&1; rc=$?; echo "occ rc=$rc"; cat gpurun_out/occ.log
  [ $rc -eq 0 ] || exit 1
fi
L=""; for x in $3; do L="$L $B/$x.so"; done
if [ -n "$L" ]; then
  timeout -k 10 500 python -u scripts/ab_probe.py $L $4 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
fi
