# Round-5 diagnostics of the general kernel's first C3 / C4-N9 launches: SQ instruction and wait
# counters (two PMC passes each) and the per-wave phase split of the -DRS_WAVELOG build.
# Usage: bash scripts/r5_diag.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag_$1; export TMPDIR=/tmp
O=gpurun_out/diag_$1; L=raft-simulation_amd/build
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
P2="SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
for wl in c3 c4_n9; do
  if [ $wl = c3 ]; then A="1048576 1"; else A="16384 1"; fi
  timeout -k 10 120 rocprofv3 --pmc $P1 -d $O/${wl}_p1 -o run -- python3 scripts/first_launch.py $wl $A $L/libraftsim.so > $O/${wl}_p1.log 2>&1 || { echo "$wl p1 failed"; tail $O/${wl}_p1.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $P2 -d $O/${wl}_p2 -o run -- python3 scripts/first_launch.py $wl $A $L/libraftsim.so > $O/${wl}_p2.log 2>&1 || { echo "$wl p2 failed"; tail $O/${wl}_p2.log; exit 1; }
  echo "$wl pmc ok"
done
timeout -k 10 300 python3 scripts/wavelog_probe.py $L/libraftsim_wavelog.so 1048576 c3 1 > $O/c3_wavelog.txt 2>&1 || { echo "wavelog c3 failed"; tail $O/c3_wavelog.txt; exit 1; }
cat $O/c3_wavelog.txt
timeout -k 10 300 python3 scripts/wavelog_probe.py $L/libraftsim_wavelog.so 16384 c4_n9 1 > $O/c4_wavelog.txt 2>&1 || { echo "wavelog c4 failed"; tail $O/c4_wavelog.txt; exit 1; }
cat $O/c4_wavelog.txt
