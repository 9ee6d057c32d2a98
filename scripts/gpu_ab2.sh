# A/B of named builds (interleaved, one process) + region counts of named diagnostic builds.
# Usage: bash scripts/gpu_ab2.sh "libA libB ..." "rclibA ..." "--c2 --c3 ..."
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
L=""; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 500 python -u scripts/ab_probe.py $L $3 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
[ $rc -eq 0 ] || exit 1
for x in $2; do
  timeout -k 10 120 python -u scripts/regioncount_probe.py $B/$x.so c2 > gpurun_out/rc_$x.log 2>&1; rc=$?; echo "rc $x $rc"; cat gpurun_out/rc_$x.log; [ $rc -eq 0 ] || exit 1
done
