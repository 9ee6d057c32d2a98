# SQ instruction / wait counters of the first launches of c2_init, C3 and C4-N9 (two PMC passes
# each, diagnostic). Usage: bash scripts/r5_pmc_first.sh TAG LIB
cd $GRAFT_REPO_ROOT; O=gpurun_out/pmcf_$1; mkdir -p $O; export TMPDIR=/tmp; LIB=$2
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
P2="SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
for wl in "c2_init 65536 1" "c3 1048576 1" "c4_n9 16384 1"; do
  set -- $wl
  timeout -k 10 120 rocprofv3 --pmc $P1 -d $O/${1}_p1 -o run -- python3 scripts/first_launch.py $1 $2 $3 $LIB > $O/${1}_p1.log 2>&1 || { echo "$1 p1 failed"; tail $O/${1}_p1.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $P2 -d $O/${1}_p2 -o run -- python3 scripts/first_launch.py $1 $2 $3 $LIB > $O/${1}_p2.log 2>&1 || { echo "$1 p2 failed"; tail $O/${1}_p2.log; exit 1; }
  echo "$1 ok"
done
