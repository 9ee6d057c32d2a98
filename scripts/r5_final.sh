# Round-5 closing run on the GPU box: the whole -m gpu suite, smoke(), and the driver's default
# bench line (written to gpurun_out/r5_bench.json).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r5_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/r5_smoke.txt; exit 1; }
cat gpurun_out/r5_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { echo "bench failed"; tail gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
