# Dynamic code-region profile (diagnostic RS_REGIONCOUNT build): per-wave execution counts of the
# tick loop's regions. Usage: bash scripts/gpu_regioncount.sh LIBNAME "c2 c3 ..."
# (build first: bash scripts/build_variants.sh rc "-DRS_REGIONCOUNT")
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
L=${1:-libraftsim_rc}
for W in ${2:-c2 c3 c4_n9}; do
  timeout -k 10 180 python -u scripts/regioncount_probe.py raft-simulation_amd/build/$L.so $W > gpurun_out/rc_$W.log 2>&1; rc=$?; echo "rc $W $rc"; cat gpurun_out/rc_$W.log; [ $rc -eq 0 ] || exit 1
done
