cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 780 python -u -m pytest tests/test_gpu_parity.py -v --timeout 240 --timeout-method thread -k "not c2_full" > gpurun_out/parity.log 2>&1; rc=$?
  echo "parity rc=$rc"
fi
if [ $rc -le 1 ]; then
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
fi
tail -5 gpurun_out/parity.log
