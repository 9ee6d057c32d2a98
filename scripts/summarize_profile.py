"""Summarize a scripts/profile.sh run (gpurun_out/prof_TAG_WL/) into profiles/ and pmc_traffic.json.

Usage: python scripts/summarize_profile.py TAG WL

Writes
  profiles/TAG_WL_kernel_stats.csv   rocprofv3 --stats of the bench run, verbatim
  profiles/TAG_WL_pmc.json           per-launch averages of every PMC counter for the tick kernel,
                                     the bench line of the profiled run, the FETCH_SIZE/WRITE_SIZE
                                     calibration and the roofline recomputed from these files alone
  profiles/TAG_fetch_calibration.json  the probe table (scripts/fetch_probe.hip)
  pmc_traffic.json                   {WL: {hbm_bytes_per_launch, kernel_src_sha, ...}} which
                                     bench.py reports as roofline.traffic when the kernel sources
                                     still hash to kernel_src_sha

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB counted at the memory
side. Rather than a blanket x2 read correction, each counter is divided by the counter-bytes-per-
true-byte ratio k that fetch_probe measured for the access shapes the tick kernel issues: its
reads are node SoA words (4 B per lane, contiguous: k_u32) and 32 B queue slots / 8 B log entries
(k_msg32), mixed in the proportion the event model assigns them (state vs message+entry bytes).
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = "tick_kernel"
# LITE launches on the steady path: the steady kernel, whose workgroups run the clusters they hand
# over through the general tick body in the same dispatch
STEADY = ("steady_lane_kernel",)


def is_steady(name):
    return any(s in name for s in STEADY)


# storm launches: the lane-per-cluster storm kernel, then the general STORM body over the clusters
# it listed (storm_kernel.hip): two dispatches, one launch
STORM = "storm_lane_kernel"


def is_tick(name):
    return is_steady(name) or KERNEL in name or STORM in name


def launch_groups(rows, name_key):
    """Dispatch-ordered rows as tick launches: one dispatch each (steady or general), or a storm
    kernel with the tick-kernel dispatch that follows it."""
    out, rerun = [], False
    for r in rows:
        name = r[name_key]
        if STORM in name:
            out.append([r])
            rerun = True
        elif is_steady(name) or KERNEL in name:
            if rerun:
                out[-1].append(r)
            else:
                out.append([r])
            rerun = False
    return out


def counters_by_kernel(path):
    """{kernel substring match -> {counter: [values per dispatch]}} from a counter_collection csv."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    rows = []
    for f in sorted(path.glob("**/*counter_collection.csv")):
        rows.extend(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))     # values in dispatch order
    for r in rows:
        out[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def calibration(src):
    spans = {}
    for line in (src / "probe_spans.txt").read_text().splitlines():
        p = line.split()
        if len(p) == 4 and p[0] == "probe":
            spans[p[1]] = (int(p[2]), int(p[3]))
    table = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for kname, vals in counters_by_kernel(src / f"cal_{ctr}").items():
            for probe, (span, req) in spans.items():
                if probe in kname and ctr in vals and (probe.startswith("rd") == (ctr == "FETCH_SIZE")):
                    b = sum(vals[ctr]) * 1024
                    table[probe] = {"counter": ctr, "counter_bytes": b, "span_bytes": span,
                                    "requested_bytes": req, "k_span": b / span,
                                    "k_requested": b / req}
    return table


def vgpr_compiler(tag, n):
    """VGPRs of the tick and steady kernel instantiations at N = n from
    profiles/TAG_kernel_resources.txt (the compiler's own counts)."""
    f = ROOT / "profiles" / f"{tag}_kernel_resources.txt"
    if not f.exists():
        return None
    return {l[:48].strip(): int(l.split()[-4]) for l in f.read_text().splitlines()
            if l.startswith((f"tick_kernel<N={n},", f"steady_lane_kernel<N={n}>"))}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r09"
    wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
    src = ROOT / "gpurun_out" / f"prof_{tag}_{wl}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    shutil.copy(src / "kt" / "run_kernel_stats.csv", dst / f"{tag}_{wl}_kernel_stats.csv")

    # the profiled run's full record (bench.py --full-json): the line on stdout is the compact one
    bench = json.loads((src / "kt_full.json").read_text())["workloads"][wl]
    pmc = collections.defaultdict(list)
    for i in range(1, 20):
        d = src / f"pmc{i}"
        if not d.exists():
            continue
        rows = []
        for f in sorted(d.glob("**/*counter_collection.csv")):
            rows.extend(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
        # one value per counter per dispatch, then summed over each launch's dispatches
        disp = collections.OrderedDict()
        for r in rows:
            if is_tick(r["Kernel_Name"]):
                e = disp.setdefault(r["Dispatch_Id"], {"Kernel_Name": r["Kernel_Name"], "c": {}})
                e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for g in launch_groups(list(disp.values()), "Kernel_Name"):
            for c in g[0]["c"]:
                pmc[c].append(sum(x["c"].get(c, 0.0) for x in g))
    # the timed launches only: the last `launches` dispatches of the tick kernel (warm-up
    # launches, on the same or a throwaway handle, come first)
    nl = max(1, bench["roofline"]["launches"])
    avg = {k: sum(v[-nl:]) / len(v[-nl:]) for k, v in pmc.items()}
    trace = list(csv.DictReader(open(src / "kt" / "run_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a launch spans its dispatches (steady kernel start to catch-up end), as the HIP events do
    groups = launch_groups(trace, "Kernel_Name")
    durs = [int(g[-1]["End_Timestamp"]) - int(g[0]["Start_Timestamp"]) for g in groups]
    stats = [r for r in csv.DictReader(open(src / "kt" / "run_kernel_stats.csv"))
             if is_tick(r["Name"])]
    durs = durs[-max(1, bench["roofline"]["launches"]):]   # the timed launches, not the warm-up
    avg_ns = sum(durs) / max(1, len(durs))

    n = bench["config"]["nodes"]
    # waves that simulate clusters: 64 // N clusters per wave on the general and wave-form steady
    # kernels, 64 per wave on the lane-per-cluster steady kernel
    lane_form = bool(groups) and any("steady_lane_kernel" in r["Kernel_Name"] for r in groups[-1])
    waves_ran = -(-bench["config"]["clusters_per_gpu"] // (64 if lane_form else 64 // n))
    cal = calibration(src)
    (dst / f"{tag}_fetch_calibration.json").write_text(json.dumps(cal, indent=1) + "\n")
    roof = bench["roofline"]
    cnt = bench["counters"]
    n = bench["config"]["nodes"]
    nodes = bench["config"]["clusters_per_gpu"] * n
    launches = max(1, roof["launches"])
    state_rd = (32 + 8 * n) * nodes
    msg_rd = (32 * cnt.get("delivered", 0) + 8 * cnt.get("entries_appended", 0)) / launches
    w_state = state_rd / max(1.0, state_rd + msg_rd)
    k_rd = w_state * cal["rd_u32_contig"]["k_span"] + (1 - w_state) * cal["rd_msg32_contig"]["k_span"]
    k_wr = w_state * cal["wr_u32_contig"]["k_span"] + (1 - w_state) * cal["wr_msg32_contig"]["k_span"]
    fetch_raw, write_raw = avg.get("FETCH_SIZE", 0) * 1024, avg.get("WRITE_SIZE", 0) * 1024
    hbm = fetch_raw / k_rd + write_raw / k_wr
    state_bytes = roof["bytes_per_launch"]           # compulsory: the hot state in and out
    event_bytes = roof["event_bytes_per_launch"]
    achieved = state_bytes / (avg_ns * 1e-9) / 1e9
    out = {
        "tag": tag, "workload": wl, "kernel_src_sha": roof["kernel_src_sha"],
        "kernel": [r["Kernel_Name"] for r in groups[-1]] if groups else None,
        "launches_traced": len(durs), "avg_duration_ns_trace": avg_ns,
        "avg_duration_ns_per_kernel_stats": {r["Name"]: float(r["AverageNs"]) for r in stats},
        "launch_note": "one dispatch per launch: the general tick kernel, or on the steady "
                       "path the steady kernel, which runs the clusters it hands over in the "
                       "same dispatch",
        "bench_avg_launch_ms_hip_events": roof["avg_launch_ms"],
        # rocprofv3's VGPR_Count field is the allocation granule count of another encoding; the
        # compiler's own register count is in profiles/TAG_kernel_resources.txt
        "vgpr_rocprof_field": {r["Kernel_Name"]: r.get("VGPR_Count") for r in groups[-1]}
        if groups else None,
        "vgpr_compiler": vgpr_compiler(tag, n),
        "pmc_per_launch": avg,
        # occupancy (MI355X_MICROARCH.md: SQ_WAVE_CYCLES in quad-cycles summed over waves;
        # GRBM_GUI_ACTIVE summed over the 8 XCDs): mean resident waves per CU over the
        # launch
        "derived": {
            "mean_waves_per_cu": 4 * avg["SQ_WAVE_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 256)
            if avg.get("GRBM_GUI_ACTIVE") and "SQ_WAVE_CYCLES" in avg else None,
            # SQ_WAVES counts every launched wave, including the waves past the packing's slots
            # in use, which exit at once (the grid covers the padded packing's bound); per-wave
            # figures divide by the waves that simulate clusters, ceil(clusters / (64 // N)), or
            # ceil(clusters / 64) for the lane-per-cluster steady kernel
            "waves_launched": avg.get("SQ_WAVES"),
            "waves_with_clusters": waves_ran,
            "valu_insts_per_wave": avg["SQ_INSTS_VALU"] / waves_ran
            if "SQ_INSTS_VALU" in avg else None,
            "salu_insts_per_wave": avg["SQ_INSTS_SALU"] / waves_ran
            if "SQ_INSTS_SALU" in avg else None,
            # SQ_LDS_BANK_CONFLICT: extra LDS cycles from conflicts (MI355X_MICROARCH.md §LDS)
            "lds_bank_conflict_per_lds_inst": avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_INSTS_LDS"]
            if avg.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in avg else None,
            # mean resident waves per SIMD over the launch: SQ_WAVE_CYCLES (quad-cycles summed
            # over waves) x 4 / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs)
            "waves_per_simd": 4 * avg["SQ_WAVE_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if avg.get("GRBM_GUI_ACTIVE") and "SQ_WAVE_CYCLES" in avg else None,
            "wait_any_frac": avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
            if avg.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in avg else None},
        "calibration": {"k_read": k_rd, "k_write": k_wr, "state_read_weight": w_state,
                        "source": f"profiles/{tag}_fetch_calibration.json"},
        "hbm_fetch_bytes_raw": fetch_raw, "hbm_write_bytes_raw": write_raw,
        "hbm_bytes_per_launch": hbm,
        "roofline_recomputed": {
            "compulsory_bytes_per_launch": state_bytes,
            "event_bytes_per_launch": event_bytes,
            "event_bytes_terms": {"state_in_out": 2 * (32 + 8 * n) * nodes,
                                  "messages_64B": 64 * cnt.get("delivered", 0) / launches,
                                  "entries_16B": 16 * cnt.get("entries_appended", 0) / launches},
            "achieved_GBs": achieved, "peak_GBs": 8000.0, "frac": achieved / 8000.0,
            "frac_event_model": event_bytes / (avg_ns * 1e-9) / 1e9 / 8000.0,
            "traffic_over_compulsory": hbm / state_bytes if state_bytes else None,
            "traffic_over_event_bytes": hbm / event_bytes if event_bytes else None,
            "how": "compulsory_bytes_per_launch / avg_duration_ns_trace (frac_event_model: the "
                   "event bytes, from the bench line's counters, bench_line below)"},
        "bench_line": bench,
    }
    (dst / f"{tag}_{wl}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    tf = ROOT / "pmc_traffic.json"
    try:
        traffic = json.loads(tf.read_text())
    except (OSError, ValueError):
        traffic = {}
    # the window the profiled bench run timed: bench.py attaches this traffic only to a line of the
    # same window (a C3 window from init-node changes cost per launch as nodes halt)
    traffic[wl] = {"hbm_bytes_per_launch": hbm, "kernel_src_sha": roof["kernel_src_sha"],
                   "window": bench.get("window"), "event_bytes_per_launch": event_bytes,
                   "compulsory_bytes_per_launch": state_bytes,
                   "traffic_over_compulsory": hbm / state_bytes if state_bytes else None,
                   "traffic_over_event_bytes": hbm / event_bytes if event_bytes else None,
                   "lds_bank_conflict_per_lds_inst":
                       out["derived"]["lds_bank_conflict_per_lds_inst"],
                   "waves_per_simd": out["derived"]["waves_per_simd"],
                   "valu_insts_per_wave": out["derived"]["valu_insts_per_wave"],
                   "source": f"profiles/{tag}_{wl}_pmc.json"}
    tf.write_text(json.dumps(traffic, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: out[k] for k in ("workload", "avg_duration_ns_trace",
                                          "bench_avg_launch_ms_hip_events", "calibration",
                                          "hbm_bytes_per_launch", "roofline_recomputed")},
                     indent=1))


if __name__ == "__main__":
    main()
