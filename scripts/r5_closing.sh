# Round-5 closing call: the -m gpu suite on the tree's library,
# the rocprofv3 passes of all eight bench workloads, smoke() and the
# default bench line. Stops at the first failure.
# Usage: bash scripts/r5_closing.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r5_gpu_tests.txt
bash scripts/profile_all.sh r5 "c2 c2_init c3 c3_spec c4_n7 c4_n9 c4_spec c5" > gpurun_out/r5_profile_all.log 2>&1 || { echo "profile failed"; tail -3 gpurun_out/r5_profile_all.log; exit 1; }
echo profiles ok
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.txt 2>&1 || { echo "smoke failed"; tail gpurun_out/r5_smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { echo "bench failed"; tail gpurun_out/r5_bench.err; exit 1; }
echo bench ok
