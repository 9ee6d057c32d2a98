# new fuzz tests, bench, profiles for the drain build
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_fuzz.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/fuzz_l.log 2>&1; rc=$?; echo "fuzz rc=$rc"; tail -3 gpurun_out/fuzz_l.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 1
bash scripts/profile.sh r10 c2 && bash scripts/profile.sh r10 c3
