# C2 wave lifetime vs cluster count (occupancy sweep), wavelog build
cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
for C in 4096 16384 32768 65536 131072; do
  timeout -k 10 120 python3 scripts/wavelog_probe.py $B/libraftsim_wavelog.so $C > gpurun_out/wl_c$C.log 2>&1 || exit 1
  echo "== $C"; head -6 gpurun_out/wl_c$C.log; tail -2 gpurun_out/wl_c$C.log
done
