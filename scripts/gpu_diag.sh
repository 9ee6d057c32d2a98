# GPU session for kernel diagnosis (never the product path): per-wave timeline of the RS_WAVELOG
# build on C2 and C3, then cost attribution of the libraftsim_cost_*.so builds against the product
# build (scripts/ab_probe.py, one process, interleaved rounds).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
timeout -k 10 180 python -u scripts/wavelog_probe.py $B/libraftsim_wl.so 65536 c2 > gpurun_out/wl_c2.log 2>&1; rc=$?; echo "wl c2 rc=$rc"; cat gpurun_out/wl_c2.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u scripts/wavelog_probe.py $B/libraftsim_wl.so 131072 c3 > gpurun_out/wl_c3.log 2>&1; rc=$?; echo "wl c3 rc=$rc"; cat gpurun_out/wl_c3.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/ab_probe.py $B/libraftsim_new.so $B/libraftsim_cost_*.so --c2 --c3 > gpurun_out/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab.log
