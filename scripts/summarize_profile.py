"""Summarize a scripts/profile.sh run (gpurun_out/prof_TAG) into profiles/TAG_*.

Writes profiles/TAG_kernel_stats.csv (rocprofv3 --stats output, verbatim), profiles/TAG_pmc.json
(per-launch averages of every PMC counter for the tick kernel) and profiles/pmc_traffic.json
(HBM bytes per tick-kernel launch for bench.py's roofline.traffic). HBM bytes follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB from the memory-side request counters;
on gfx950 FETCH_SIZE reads half the bytes of wide coalesced streaming reads, so both the raw value
and the x2-corrected read side are recorded (this kernel's reads are narrow gathers, for which the
guide gives no calibration; the write side dominates here).
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = ROOT / "gpurun_out" / f"prof_{tag}"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
shutil.copy(src / "kt" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
pmc = collections.defaultdict(list)
for f in sorted(src.glob("pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "tick_kernel" in r["Kernel_Name"]:
            pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in pmc.items()}
trace = list(csv.DictReader(open(src / "kt" / "run_kernel_trace.csv")))
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace
        if "tick_kernel" in r["Kernel_Name"]]
fetch, write = avg.get("FETCH_SIZE", 0) * 1024, avg.get("WRITE_SIZE", 0) * 1024
out = {"tag": tag, "kernel": "rs::tick_kernel<5>", "launches_profiled": len(durs),
       "avg_duration_ns": sum(durs) / max(1, len(durs)),
       "vgpr": next((r.get("VGPR_Count") for r in trace if "tick_kernel" in r["Kernel_Name"]), None),
       "pmc_per_launch": avg,
       "hbm_fetch_bytes_raw": fetch, "hbm_write_bytes": write,
       "hbm_bytes_per_launch": 2 * fetch + write,
       "note": "2*FETCH_SIZE + WRITE_SIZE per the gfx950 FETCH_SIZE correction; see docstring"}
(dst / f"{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
(dst / "pmc_traffic.json").write_text(json.dumps(
    {"source": f"profiles/{tag}_pmc.json", "hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
     "workload": "C2 bench, 10,000 ticks per launch"}, indent=1) + "\n")
print(json.dumps(out, indent=1))
