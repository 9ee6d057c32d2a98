# BASELINE configs 3-5 on one MI355X next to the CPU oracle (scripts/bench_configs.py).
# Usage: bash scripts/gpu_configs.sh TAG
TAG=${1:-r14}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for C in c3 c4 c5; do
  timeout -k 10 500 python -u scripts/bench_configs.py $C >> gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$C.err || { echo "$C failed"; tail gpurun_out/configs_$C.err; exit 1; }
  echo "$C ok"
done
cat gpurun_out/configs_$TAG.jsonl
