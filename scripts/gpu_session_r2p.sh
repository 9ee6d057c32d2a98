# bench under torch.distributed.run (RCCL path at world size 1) and the default bench
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_trun.json 2> gpurun_out/bench_trun.err; rc=$?; echo "torchrun rc=$rc"; tail -c 600 gpurun_out/bench_trun.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_trun.err; exit 1; }
