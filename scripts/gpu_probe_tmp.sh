cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_probe scripts/launch_probe.hip > /dev/null 2>&1 || { echo "probe build failed"; exit 1; }
timeout -k 10 60 /tmp/launch_probe > gpurun_out/launch_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/launch_probe.txt
