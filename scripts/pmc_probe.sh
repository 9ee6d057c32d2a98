# PMC passes (each its own run, <= 8 SQ counters) over scripts/run_c2.py for one build.
# Usage: bash scripts/pmc_probe.sh LIBNAME OUTTAG [KERNEL-NAME-SUBSTRING (default tick_kernel)]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_$2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
KN=${3:-tick_kernel}
for PMC in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVES" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/run_c2.py $R/raft-simulation_amd/build/$1.so > $OUT/p$i.log 2>&1 || { echo "pmc$i failed $?"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pmc$i ok"
done
python3 - $OUT $KN <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id") or 0))
    for r in rows:
        if sys.argv[2] in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    v = v[-5:]
    print(f"{k:32s} {sum(v) / len(v):16.0f}")
PY
