# C3 from init, per-launch kernel times for named builds (scripts/c3_window.py)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
L=""; for x in $3; do L="$L $B/$x.so"; done
timeout -k 10 600 python -u scripts/c3_window.py $1 $2 $L > gpurun_out/c3w.log 2>&1; rc=$?; echo "c3w rc=$rc"; cat gpurun_out/c3w.log
