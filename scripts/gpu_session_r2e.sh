cd $GRAFT_REPO_ROOT; B=raft-simulation_amd/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu -q -x --timeout 300 --timeout-method thread -k "schedule or c2_small or c3_faults or spec_c3 or tiny or shard or multi_launch or step_async or n2 or n8 or kat" > gpurun_out/quick6.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/quick6.log
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_base.so $B/libraftsim_new.so --c2 --c3 --rounds=8
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kt11 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --steps 12 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/kt11.log 2>&1; echo "kt rc=$?"
