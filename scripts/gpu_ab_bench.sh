# A/B of kernel builds on the bench workloads themselves (bench.py, RAFTSIM_LIB selects the build),
# then scripts/ab_probe.py over the same builds. Usage: bash scripts/gpu_ab_bench.sh WORKLOAD
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
WL=${1:-c3}
for L in raft-simulation_amd/build/libraftsim*.so; do
  RAFTSIM_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abb_$(basename $L .so).json 2> gpurun_out/abb.err || { echo "bench $L failed"; tail -5 gpurun_out/abb.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w=d.get('workloads',{}).get('$WL',d); print('$L', '$WL', 'ms/step', round(w['ms_per_step'],3), 'kernel', round(w['roofline']['avg_launch_ms'],3), 'value %.3e' % w['value'])" gpurun_out/abb_$(basename $L .so).json
done
timeout -k 10 400 python -u scripts/ab_probe.py raft-simulation_amd/build/libraftsim*.so --c3 --c4_n9 > gpurun_out/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab.log
