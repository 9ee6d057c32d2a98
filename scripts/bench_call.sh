# gpurun wrapper: the driver-default bench line into gpurun_out/TAG_bench.json (+ _full.json) and its summary
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 600 python bench.py --full-json gpurun_out/$1_bench_full.json > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err; rc=$?; python scripts/bench_summary.py gpurun_out/$1_bench.json; exit $rc
