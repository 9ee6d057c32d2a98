# One call for the round's measurements: A/B of the steady kernel forms, the round-end session
# (smoke, -m gpu suite, bench, C3 warm-up check, torchrun) and the C2 rocprofv3 profile.
# Usage: bash scripts/gpu_round.sh TAG
TAG=${1:-r22}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=raft-simulation_amd/build
if [ -f $B/libraftsim_old.so ]; then
  timeout -k 10 200 python -u scripts/ab_probe.py $B/libraftsim.so $B/libraftsim_old.so --c2 --rounds=9 > gpurun_out/ab_round.log 2>&1 || { echo "ab failed"; tail gpurun_out/ab_round.log; exit 1; }
  cat gpurun_out/ab_round.log
fi
bash scripts/gpu_session.sh $TAG || exit 1
bash scripts/profile.sh $TAG c2 || exit 1
echo "round measurements ok"
