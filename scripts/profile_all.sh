# rocprofv3 passes over bench.py workloads (the driver's window: 20 steps, 5 warm-up): a kernel
# trace + stats run, then FETCH_SIZE and WRITE_SIZE each in a run of their own, one SQ pass
# (occupancy, LDS bank conflicts, instruction mix), and with FULL=1 a second, diagnostic SQ pass
# (wait and issue breakdown); once per call the FETCH/WRITE calibration
# probe (scripts/fetch_probe.hip). Every step under its own time limit, steps chained: the first
# failure ends the script.
# Usage: bash scripts/profile_all.sh TAG "c2 c2_init c3 ..."      (outputs gpurun_out/prof_TAG_WL/)
set -u
TAG=$1
WLS=$2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
PROBE=/tmp/fetch_probe_$$
hipcc --offload-arch=gfx950 -O3 -o $PROBE $R/scripts/fetch_probe.hip > /tmp/probe_build.log 2>&1 || { echo "probe build failed"; exit 1; }
for WL in $WLS; do
  OUT=$R/gpurun_out/prof_${TAG}_${WL}
  mkdir -p $OUT
  B="$R/bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $B --full-json $OUT/kt_full.json > $OUT/kt.log 2>&1 || { echo "$WL kt failed $?"; exit 1; }
  echo "$WL kt ok"
  i=0
  for PMC in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 $B > $OUT/pmc$i.log 2>&1 || { echo "$WL pmc$i failed $?"; exit 1; }
    echo "$WL pmc$i ok"
  done
  if [ "${FULL:-0}" = 1 ]; then
    for PMC in "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 400 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 $B > $OUT/pmc$i.log 2>&1 || { echo "$WL pmc$i failed $?"; exit 1; }
      echo "$WL pmc$i ok"
    done
  fi
  $PROBE > $OUT/probe_spans.txt 2>&1 || { echo "probe failed $?"; exit 1; }
  for PMC in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $PMC --output-format csv -d $OUT/cal_$PMC -o run -- $PROBE > $OUT/cal_$PMC.log 2>&1 || { echo "cal $PMC failed $?"; exit 1; }
  done
  echo "$WL cal ok"
done
