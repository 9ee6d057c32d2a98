"""bench.py's host logic on the CPU (no GPU run): the workload table covers every BASELINE config,
the compulsory-byte roofline arithmetic, the tick windows, and the rule that PMC traffic is
attached to a line only when it was measured on the same kernel sources over the same window."""
import importlib.util
import json
from pathlib import Path
from types import SimpleNamespace

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_default_workloads_cover_the_baseline_configs(bench):
    """BASELINE.json configs 2-5 (config 1 is the reference's CPU case: the c1 golden trace)."""
    default = None
    src = (ROOT / "bench.py").read_text()
    for line in src.splitlines():
        if '"--workload"' in line:
            default = line.split('default="', 1)[1].split('"', 1)[0]
    assert default is not None
    names = default.split("+")
    assert names[0] == "c2"                      # the headline line is config 2
    assert {"c2", "c2_init", "c3", "c3_spec", "c4_n7", "c4_n9", "c4_spec", "c5"} <= set(names)
    assert all(n in bench.WORKLOADS for n in names)
    w = bench.WORKLOADS
    assert w["c2"]["clusters"] == 65536 and w["c2"]["cfg"]["nodes"] == 5
    assert w["c3"]["clusters"] == 1 << 20 and w["c3"]["cfg"]["drop_ppm"] == 100000
    # config 4: 7- and 9-node clusters with 4096-entry logs, from init-node (the replication
    # and its 1000+-entry AppendEntries are inside the window), and its Spec-Raft form (the
    # commit index by the sorting network)
    for name, nodes in (("c4_n7", 7), ("c4_n9", 9), ("c4_spec", 9)):
        assert w[name]["cfg"]["nodes"] == nodes and w[name]["cfg"]["log_cap"] == 4096
        assert w[name]["window"] == "init"
    assert w["c4_spec"]["cfg"]["variant_flags"] == 2
    assert w["c5"]["cfg"]["variant_flags"] & 1 and w["c5"]["window"] == "violation"


def test_roofline_is_compulsory_bytes_over_launch_time(bench):
    spec = bench.WORKLOADS["c2"]
    delta = {"delivered": 1_000_000, "entries_appended": 0}
    r = bench.roofline("c2", spec, 65536, 5, 20, 0.025, delta, {"kind": "none"}, 1)
    state = 2 * (32 + 8 * 5) * 65536 * 5             # S_node = 32 + 8N bytes, in and out once
    assert r["bytes_per_launch"] == state
    assert r["achieved"] == pytest.approx(state / 25e-6 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS)
    # the event model adds 64 B per delivered message (per launch over all ranks' launches)
    assert r["event_bytes_per_launch"] == pytest.approx(state + 64 * 1_000_000 / 20)
    assert r["frac_event_model"] > r["frac"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert r["traffic"] is None                       # no profile of window "none"


def test_default_warmup_is_the_drivers(bench):
    """The driver runs `bench.py --steps 20 --warmup 5`: the defaults are that window, so the
    PMC profiles taken with the defaults describe the driver's window."""
    src = (ROOT / "bench.py").read_text()
    assert 'ap.add_argument("--warmup", type=int, default=5)' in src
    assert 'ap.add_argument("--steps", type=int, default=20)' in src


def test_survey_8d_accounting(bench):
    d = {"node_ticks": 10 ** 9, "delivered": 0, "entries_appended": 0}
    r = bench.survey_8d(1e14, 5, d)
    assert r["bytes_per_node_tick"] == 152                  # B(5) with m = e = 0
    assert r["value"] == pytest.approx(1e14 * 152 / 8e12)


def test_windows(bench):
    args = SimpleNamespace(steps=20, warmup=2)
    assert bench.window_id(bench.WORKLOADS["c2"], args) == {"kind": "steady", "steps": 20,
                                                             "warmup": 2}
    assert bench.window_id(bench.WORKLOADS["c3"], args) == {"kind": "init", "steps": 20}
    assert bench.window_id(bench.WORKLOADS["c2_init"], args) == {"kind": "first", "steps": 1}
    assert bench.window_id(bench.WORKLOADS["c5"], args)["kind"] == "violation"


def test_traffic_only_from_the_same_sources_and_window(bench, tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    for f in bench.KERNEL_SOURCES:
        p = tmp_path / f
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("kernel source " + f)
    sha = bench.kernel_build_hash()
    win = {"kind": "steady", "steps": 20, "warmup": 2}
    rec = {"c2": {"kernel_src_sha": sha, "window": win, "hbm_bytes_per_launch": 123.0,
                  "source": "profiles/x.json"}}
    (tmp_path / "pmc_traffic.json").write_text(json.dumps(rec))
    assert bench.load_traffic("c2", win) == (123.0, "profiles/x.json")
    assert bench.load_traffic("c2", dict(win, steps=5))[0] is None        # another window
    assert bench.load_traffic("c3", win)[0] is None                        # no profile
    (tmp_path / bench.KERNEL_SOURCES[0]).write_text("edited")              # another build
    assert bench.load_traffic("c2", win) == (None, "PMC profile of another kernel build")



def _worst_case_record(bench, name, world):
    """A record shaped like run_workload's, every field present and every float at full
    precision, with long prose and a full counter dict (the round-5 line was 24 KB of these)."""
    spec = bench.WORKLOADS[name]
    long = "x" * 400
    counters = {f"counter_{i}": 123456789012345 + i for i in range(40)}
    roof = {k: 0.123456789012345 for k in ("achieved", "frac", "frac_measured", "traffic",
                                           "traffic_over_compulsory", "avg_launch_ms",
                                           "lds_bank_conflict_per_lds_inst", "waves_per_simd",
                                           "frac_event_model", "event_bytes_per_launch")}
    roof.update(bound="hbm", peak=8000.0, unit="GB/s", bytes_per_launch=755000000,
                model=bench.MODEL["general"], traffic_source=long, avg_launch_source=long,
                limiter=long, kernel_src_sha="0" * 16, launches=20,
                survey_8d={"value": 1.0, "note": long})
    rec = {"value": 3.901234567890123e14, "unit": "node-ticks/s", "ms_per_step": 0.00841234567,
           "wall_ms_per_step": 0.123456789, "wall_value": 1.23456789e13, "timing": long,
           "scaling": spec["scaling"], "window": {"kind": "init", "steps": 20},
           "config": {"workload": spec["desc"], "clusters": spec["clusters"] * world,
                      "clusters_per_gpu": spec["clusters"], "nodes": spec["cfg"]["nodes"],
                      "ticks_per_step": 10000, "parallelism": f"cluster-sharded x{world}"},
           "roofline": roof, "events_per_s": 2.4123456789e11, "live_node_frac_end": 0.15812345,
           "live_node_ticks_per_s": 6.9812345e10, "payload_evicted": 0, "ev_ae": 655360,
           "payload_max": 2156, "counters": counters, "timed_launch_ms": 0.008123456,
           "timed_launches": 1, "first_violation_tick": 16572, "time_to_first_violation_s": 0.015,
           "cpu_baseline": {"value": 1.8912345e11, "unit": "node-ticks/s", "cores": 16,
                            "kind": "port", "sample": long, "short_sample": "y" * 90,
                            "host_cpus": {"affinity": 16}, "every_tick_value": 1.5e9,
                            "every_tick_sample": long, "bit_exact": True}}
    return rec


@pytest.mark.parametrize("world", [1, 8])
def test_bench_line_fits_the_drivers_tail(bench, world):
    """the driver keeps ~8,000 characters of stdout and parses the last line,
    so the one JSON line must stay well under that with every workload on it; the headline keys,
    roofline and cpu_baseline are on it and n_gpus / parallelism follow the world size."""
    src = (ROOT / "bench.py").read_text()
    default = next(l.split('default="', 1)[1].split('"', 1)[0] for l in src.splitlines()
                   if '"--workload"' in l)
    names = default.split("+")
    recs = {n: _worst_case_record(bench, n, world) for n in names}
    args = SimpleNamespace(steps=20, warmup=5)
    out = bench.compact_line(names, recs, world, args, str(ROOT / "gpurun_out" / "bench_full.json"))
    line = json.dumps(out)
    assert len(line) < 6000, len(line)
    assert "\n" not in line
    back = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline",
              "cpu_baseline", "workloads"):
        assert k in back, k
    assert back["n_gpus"] == world
    assert back["config"]["parallelism"] == f"cluster-sharded x{world}"
    for k in ("frac", "achieved", "peak", "traffic", "frac_measured",
              "lds_bank_conflict_per_lds_inst", "waves_per_simd", "model"):
        assert k in back["roofline"], k
    assert {"value", "cores", "kind"} <= set(back["cpu_baseline"])
    assert set(back["workloads"]) == set(names[1:])
    for w in back["workloads"].values():
        assert {"value", "ms_per_step", "frac", "traffic", "cpu"} <= set(w)
    assert back["full_record"] == "gpurun_out/bench_full.json"


def test_pmc_record_feeds_occupancy_and_conflicts(bench, tmp_path, monkeypatch):
    """roofline carries the same-sha profile's LDS bank conflicts and waves per SIMD, and
    frac_measured = PMC bytes / launch time / peak beside the compulsory frac."""
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    for f in bench.KERNEL_SOURCES:
        p = tmp_path / f
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("kernel source " + f)
    win = {"kind": "steady", "steps": 20, "warmup": 5}
    rec = {"c2": {"kernel_src_sha": bench.kernel_build_hash(), "window": win,
                  "hbm_bytes_per_launch": 25.6e6, "source": "profiles/x.json",
                  "lds_bank_conflict_per_lds_inst": 0.01, "waves_per_simd": 0.9}}
    (tmp_path / "pmc_traffic.json").write_text(json.dumps(rec))
    r = bench.roofline("c2", bench.WORKLOADS["c2"], 65536, 5, 20, 0.008, {"delivered": 0,
                       "entries_appended": 0}, win, 1)
    assert r["frac_measured"] == pytest.approx(25.6e6 / 8e-6 / 1e9 / 8000)
    assert r["lds_bank_conflict_per_lds_inst"] == 0.01 and r["waves_per_simd"] == 0.9
    assert "Infinity-Cache" in r["model"]
