# A/B of named builds only (scripts/ab_probe.py). Usage: bash scripts/gpu_ab_only.sh "libA libB ..." "--c2 ..."
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
L=""; for x in $1; do L="$L $B/$x.so"; done
timeout -k 10 500 python -u scripts/ab_probe.py $L $2 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
