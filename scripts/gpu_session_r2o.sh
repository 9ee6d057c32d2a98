# client gap with the table read up front, power-of-two period/burst by shifts
cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/suite_o.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/suite_o.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u scripts/ab_probe.py $B/libraftsim_base.so $B/libraftsim_new.so --c2 --c3 --c4_n9 --rounds=6 || exit 1
