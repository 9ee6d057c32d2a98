# GPU session: smoke, the whole -m gpu suite, bench (N=1 with CPU baseline) and the torchrun/RCCL path.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
fi
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
fi
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_dist.log 2>&1; echo "bench_dist rc=$?"
fi
