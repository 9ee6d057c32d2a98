# rocprofv3 kernel trace + stats of scripts/run_c2.py for each named build (diagnostic).
# Usage: bash scripts/gpu_kt.sh "libA libB"
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for x in $1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_$x -o run -- python3 $R/scripts/run_c2.py $R/raft-simulation_amd/build/$x.so > $R/gpurun_out/kt_$x.log 2>&1 || { echo "kt $x failed $?"; exit 1; }
  echo "== $x"; cat $R/gpurun_out/kt_$x.log | tail -2
  cat $(find $R/gpurun_out/kt_$x -name "*kernel_stats.csv") | cut -c1-220
done
