# client-sets to halted nodes skipped
cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/suite_n.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/suite_n.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_base.so $B/libraftsim_new.so --c2 --c3 --c4_n9 --rounds=4 || exit 1
timeout -k 10 200 python3 scripts/wavelog_probe.py $B/libraftsim_wavelog.so 131072 c3 > gpurun_out/wl_c3n.log 2>&1; echo "wl rc=$?"; grep "kernel_ms\|active ticks\|injection" gpurun_out/wl_c3n.log
