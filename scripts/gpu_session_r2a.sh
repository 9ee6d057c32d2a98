# Round-2 GPU session A: full GPU suite, occupancy sweep, A/B of residency variants, counter list.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAILED|^E  " gpurun_out/gpu_tests4.log | head -20
timeout -k 10 200 python -u scripts/occ_probe.py 24576 36864 45000 49152 53248 57344 61440 65536 > gpurun_out/occ.log 2>&1 && echo "occ ok" && cat gpurun_out/occ.log && \
timeout -k 10 400 python -u scripts/ab_probe.py raft-simulation_amd/build/libraftsim_base.so raft-simulation_amd/build/libraftsim_nohbm.so raft-simulation_amd/build/libraftsim_nohbm_w5.so raft-simulation_amd/build/libraftsim_w5.so --c2 --c3 --rounds=6 > gpurun_out/ab.log 2>&1 && echo "ab ok" && cat gpurun_out/ab.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
