cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/footprint_probe.py > gpurun_out/footprint.log 2>&1; echo "fp rc=$?"; cat gpurun_out/footprint.log
bash scripts/profile.sh r09 c2
