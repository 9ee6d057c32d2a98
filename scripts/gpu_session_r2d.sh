cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "schedule or c2_small or c3_faults or spec_c3 or tiny or shard or multi_launch or step_async" > gpurun_out/quick5.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/quick5.log
timeout -k 10 120 python -u scripts/wavelog_probe.py $B/libraftsim_wavelog.so 65536 || exit 1
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_base.so $B/libraftsim_new.so --c2 --c3 --c4_n9 --rounds=8
