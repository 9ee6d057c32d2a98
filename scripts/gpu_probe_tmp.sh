cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/lane_timeline.py raft-simulation_amd/build/libraftsim_wavelog.so 65536 6 > gpurun_out/timeline.txt 2>&1 || { echo "timeline failed"; tail gpurun_out/timeline.txt; exit 1; }
cat gpurun_out/timeline.txt
timeout -k 10 300 python bench.py --workload c2+c4_n9 --no-cpu-baseline > gpurun_out/bench_c2c4.json 2> gpurun_out/bench_c2c4.err || { echo "bench failed"; tail gpurun_out/bench_c2c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2c4.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']); w=d['workloads']['c4_n9']; print(w['value'], w['ms_per_step'], w['roofline']['avg_launch_ms'])"
