# rocprofv3 passes over the bench: kernel trace + stats, then one PMC group per pass (each pass its
# own run, counter limits per block respected: <=8 SQ, <=4 TCC, <=4 TCP, <=2 TA, <=2 GRBM).
# Usage: bash scripts/profile.sh TAG [WORKLOAD]   (outputs gpurun_out/prof_TAG_WORKLOAD/)
set -u
TAG=${1:-r09}
WL=${2:-c2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# the bench defaults (20 steps, 5 warm-up): the same window as the driver's bench line
B="$R/bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $B > $OUT/kt.log 2>&1 || { echo "kt failed $?"; exit 1; }
echo "kt ok"
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_INSTS_SMEM SQ_WAIT_INST_LDS" \
           "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_TCC_READ_REQ" \
           "TCP_TCC_READ_REQ_LATENCY TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_WRITE_REQ TCP_PENDING_STALL_CYCLES" \
           "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 $B > $OUT/pmc$i.log 2>&1 || { echo "pmc$i failed $?"; exit 1; }
  echo "pmc$i ok"
done
# FETCH_SIZE / WRITE_SIZE calibration over known byte counts (scripts/fetch_probe.hip)
PROBE=/tmp/fetch_probe_$$
hipcc --offload-arch=gfx950 -O3 -o $PROBE $R/scripts/fetch_probe.hip > $OUT/probe_build.log 2>&1 || { echo "probe build failed"; exit 1; }
$PROBE > $OUT/probe_spans.txt 2>&1 || { echo "probe failed $?"; exit 1; }
for PMC in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $PMC --output-format csv -d $OUT/cal_$PMC -o run -- $PROBE > $OUT/cal_$PMC.log 2>&1 || { echo "cal $PMC failed $?"; exit 1; }
  echo "cal $PMC ok"
done
