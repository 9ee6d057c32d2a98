"""scripts/summarize_profile.py on a synthetic rocprofv3 output tree (CPU): the per-launch PMC
averages over the timed launches, the FETCH/WRITE calibration, the SQ-derived occupancy and LDS
bank-conflict figures, and the pmc_traffic.json record bench.py attaches to its line (VERDICT r5
items 3-4: the north-star counters on the line, from same-source profiles)."""
import csv
import importlib.util
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _mod():
    spec = importlib.util.spec_from_file_location("summarize_under_test",
                                                  ROOT / "scripts" / "summarize_profile.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _csv(path, rows):
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_summary_derives_occupancy_conflicts_and_traffic(tmp_path, monkeypatch):
    m = _mod()
    monkeypatch.setattr(m, "ROOT", tmp_path)
    src = tmp_path / "gpurun_out" / "prof_T_c4_n9"
    kname = "void rs::tick_kernel<9, false, false, false, false>(rs::DevSim, unsigned int, unsigned int)"
    launches = 3
    # one warm-up dispatch, then the three timed launches, 1 ms apart, each 0.5 ms long
    trace = [{"Kernel_Name": kname, "Start_Timestamp": str(i * 1_000_000),
              "End_Timestamp": str(i * 1_000_000 + 500_000)} for i in range(launches + 1)]
    _csv(src / "kt" / "run_kernel_trace.csv", trace)
    _csv(src / "kt" / "run_kernel_stats.csv", [{"Name": kname, "AverageNs": "500000"}])
    full = {"workloads": {"c4_n9": {
        "roofline": {"launches": launches, "bytes_per_launch": 1_000_000, "avg_launch_ms": 0.5,
                     "event_bytes_per_launch": 2_000_000, "kernel_src_sha": "abc"},
        "counters": {"delivered": 0, "entries_appended": 0},
        "config": {"nodes": 9, "clusters_per_gpu": 16384}, "window": {"kind": "init", "steps": 3}}}}
    (src / "kt_full.json").write_text(json.dumps(full))

    def pmc(i, counters):
        rows = []
        for d in range(launches + 1):
            for c, v in counters.items():
                rows.append({"Dispatch_Id": str(d), "Kernel_Name": kname, "Counter_Name": c,
                             "Counter_Value": str(v * (100 if d == 0 else 1))})
        _csv(src / f"pmc{i}" / "run_counter_collection.csv", rows)

    pmc(1, {"FETCH_SIZE": 1000})                 # KiB
    pmc(2, {"WRITE_SIZE": 500})
    pmc(3, {"SQ_WAVES": 2341, "SQ_WAVE_CYCLES": 2_000_000, "SQ_INSTS_LDS": 1000,
            "SQ_LDS_BANK_CONFLICT": 250, "SQ_WAIT_ANY": 800_000, "SQ_INSTS_VALU": 2341 * 500,
            "SQ_INSTS_SALU": 10, "SQ_BUSY_CYCLES": 1, "GRBM_GUI_ACTIVE": 8 * 1000})
    (src / "probe_spans.txt").write_text("probe rd_u32_contig 1000 1000\nprobe rd_msg32_contig 1000 1000\n"
                                         "probe wr_u32_contig 1000 1000\nprobe wr_msg32_contig 1000 1000\n")
    for ctr, probes, kib in (("FETCH_SIZE", ("rd_u32_contig", "rd_msg32_contig"), 0.5 * 1000 / 1024),
                             ("WRITE_SIZE", ("wr_u32_contig", "wr_msg32_contig"), 1000 / 1024)):
        _csv(src / f"cal_{ctr}" / "run_counter_collection.csv",
             [{"Dispatch_Id": str(j), "Kernel_Name": f"probe_{p}", "Counter_Name": ctr,
               "Counter_Value": str(kib)} for j, p in enumerate(probes)])
    monkeypatch.setattr(sys, "argv", ["summarize_profile.py", "T", "c4_n9"])
    m.main()
    rec = json.loads((tmp_path / "pmc_traffic.json").read_text())["c4_n9"]
    # timed launches only (the 100x warm-up dispatch is dropped); FETCH_SIZE counts 0.5 of the
    # bytes read (calibration), WRITE_SIZE 1.0
    assert rec["hbm_bytes_per_launch"] == pytest.approx(1000 * 1024 / 0.5 + 500 * 1024)
    assert rec["lds_bank_conflict_per_lds_inst"] == pytest.approx(0.25)
    # 4 x quad-cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs)
    assert rec["waves_per_simd"] == pytest.approx(4 * 2_000_000 / (1000 * 1024))
    assert rec["valu_insts_per_wave"] == pytest.approx(500)
    assert rec["kernel_src_sha"] == "abc" and rec["window"] == {"kind": "init", "steps": 3}
    out = json.loads((tmp_path / "profiles" / "T_c4_n9_pmc.json").read_text())
    assert out["avg_duration_ns_trace"] == pytest.approx(500_000)
    assert out["derived"]["wait_any_frac"] == pytest.approx(0.4)
