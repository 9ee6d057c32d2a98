# C3 burst-step diagnostics: per-wave phase split (-DRS_WAVELOG build) of the bench window's
# launches 2-4 from init-node (ticks [10k, 40k)), the burst launches included.
# Usage: bash scripts/r5_diag3.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag_$1; O=gpurun_out/diag_$1; L=raft-simulation_amd/build
for k in 2 3 4; do
  timeout -k 10 300 python3 scripts/wavelog_probe.py $L/libraftsim_wavelog.so 1048576 c3 $k > $O/c3_wavelog_$k.txt 2>&1 || { echo "wavelog c3 $k failed"; tail $O/c3_wavelog_$k.txt; exit 1; }
  echo "== c3 step $k"; cat $O/c3_wavelog_$k.txt
done
