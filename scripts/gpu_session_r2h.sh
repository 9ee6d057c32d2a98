# residency: VGPR-capped 5/6 waves per SIMD with next/match in the cluster block (LDS 6.6 KB)
cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 120 python3 scripts/wavelog_probe.py $B/libraftsim_wavelog.so > gpurun_out/wl_h.log 2>&1; echo "wl rc=$?"; tail -2 gpurun_out/wl_h.log
timeout -k 10 500 python -u scripts/ab_probe.py $B/libraftsim_new.so $B/libraftsim_nm0.so $B/libraftsim_w5nm0.so $B/libraftsim_w6nm0.so --c2 --c3 --c4_n9 --rounds=6 || exit 1
