# Diagnostic GPU session (never the product path): per-wave timeline of the RS_WAVELOG build on C2,
# the occupancy sweep of the product build, and a short C2 bench line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
TAG=${1:-base}
timeout -k 10 180 python -u scripts/wavelog_probe.py $B/libraftsim_wl.so 65536 c2 > gpurun_out/wl_c2_$TAG.log 2>&1; rc=$?; echo "wl rc=$rc"; cat gpurun_out/wl_c2_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u scripts/occ_probe.py > gpurun_out/occ_$TAG.log 2>&1; rc=$?; echo "occ rc=$rc"; cat gpurun_out/occ_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2>&1; rc=$?; echo "bench rc=$rc"; head -c 600 gpurun_out/bench_$TAG.json
