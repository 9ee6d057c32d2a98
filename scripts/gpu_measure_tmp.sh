cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/lane_timeline.py raft-simulation_amd/build/libraftsim_wavelog.so 65536 6 > gpurun_out/timeline.txt 2>&1 || { echo "timeline failed"; tail gpurun_out/timeline.txt; exit 1; }
cat gpurun_out/timeline.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -30 gpurun_out/bench_full.err; exit 1; }
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kt_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/kt_c2.log 2>&1 || { echo "kt failed"; exit 1; }
echo kt ok
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/wavelog_probe.py raft-simulation_amd/build/libraftsim_wavelog.so 131072 c3 4 > gpurun_out/wl_c3.txt 2>&1 || { echo "wl c3 failed"; tail gpurun_out/wl_c3.txt; exit 1; }
cat gpurun_out/wl_c3.txt
timeout -k 10 200 python -u scripts/wavelog_probe.py raft-simulation_amd/build/libraftsim_wavelog.so 131072 c3_spec 4 > gpurun_out/wl_c3s.txt 2>&1 || { echo "wl c3s failed"; tail gpurun_out/wl_c3s.txt; exit 1; }
cat gpurun_out/wl_c3s.txt
cd $GRAFT_REPO_ROOT
hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_probe scripts/launch_probe.hip > /dev/null 2>&1 || { echo "probe build failed"; exit 1; }
timeout -k 10 60 /tmp/launch_probe > gpurun_out/launch_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/launch_probe.txt
timeout -k 10 120 python scripts/dispatch_probe.py raft-simulation_amd/build/libraftsim.so raft-simulation_amd/build/libraftsim_loadonly.so > gpurun_out/dispatch_probe.txt 2>&1 || { echo "dprobe failed"; tail gpurun_out/dispatch_probe.txt; exit 1; }
cat gpurun_out/dispatch_probe.txt
