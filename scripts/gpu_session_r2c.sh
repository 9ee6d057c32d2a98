cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
for v in wavelog wavelogkt; do echo "== $v"; timeout -k 10 120 python -u scripts/wavelog_probe.py $B/libraftsim_$v.so 65536 || exit 1; done
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_base.so $B/libraftsim_keytimer.so --c2 --c3 --c4_n9 --rounds=8
