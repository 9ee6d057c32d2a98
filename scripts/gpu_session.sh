# Round-end style GPU session: smoke, the whole -m gpu suite, the bench (N=1 with CPU baseline),
# the C3 window with another warm-up (warm-up independence), the torchrun/RCCL path at world size 1.
# Usage: bash scripts/gpu_session.sh TAG      (profiles: scripts/profile.sh TAG WORKLOAD)
TAG=${1:-r21}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
echo "smoke ok"; cat gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
echo "bench ok"
timeout -k 10 300 python bench.py --workload c3 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_c3w5.json 2> gpurun_out/bench_w5.err || { echo "bench w5 failed"; tail gpurun_out/bench_w5.err; exit 1; }
echo "bench c3 warmup 5 ok"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/bench_dist.log 2>&1 || { echo "torchrun bench failed"; tail gpurun_out/bench_dist.log; exit 1; }
echo "torchrun bench ok"
