# NM_LDS off (next/match in the cluster block, LDS 9.2 -> 6.6 KB per wave: 17 -> 24 waves per CU)
cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_new.so $B/libraftsim_nm0.so --c2 --c3 --c4_n9 --rounds=6 || exit 1
