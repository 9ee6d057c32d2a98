cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for W in c2 c3 c4_n9; do
  timeout -k 10 180 python -u scripts/regioncount_probe.py raft-simulation_amd/build/libraftsim_rc.so $W > gpurun_out/rc_$W.log 2>&1; rc=$?; echo "rc $W $rc"; cat gpurun_out/rc_$W.log; [ $rc -eq 0 ] || exit 1
done
