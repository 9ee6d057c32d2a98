# c2_init diagnostics: per-wave phase split of the first 10k-tick launch from init-node
# (-DRS_WAVELOG build) and the launch split probe.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag_$1; O=gpurun_out/diag_$1; L=raft-simulation_amd/build
timeout -k 10 120 python3 scripts/wavelog_probe.py $L/libraftsim_wavelog.so 65536 c2 1 > $O/c2_wavelog.txt 2>&1 || { echo "wavelog c2 failed"; tail $O/c2_wavelog.txt; exit 1; }
cat $O/c2_wavelog.txt
