# Per-wave timelines (RS_WAVELOG builds) at several cluster counts: bash scripts/gpu_wl.sh "libs" "counts"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
for w in $1; do for c in $2; do
  timeout -k 10 180 python -u scripts/wavelog_probe.py $B/$w.so $c c2 > gpurun_out/wl_${w}_$c.log 2>&1; rc=$?; echo "== wl $w $c rc=$rc"; cat gpurun_out/wl_${w}_$c.log
  [ $rc -eq 0 ] || exit 1
done; done
