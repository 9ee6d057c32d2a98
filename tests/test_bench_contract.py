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
    assert {"c2", "c2_init", "c3", "c3_spec", "c4_n9", "c5"} <= set(names)
    assert all(n in bench.WORKLOADS for n in names)
    w = bench.WORKLOADS
    assert w["c2"]["clusters"] == 65536 and w["c2"]["cfg"]["nodes"] == 5
    assert w["c3"]["clusters"] == 1 << 20 and w["c3"]["cfg"]["drop_ppm"] == 100000
    assert w["c4_n9"]["cfg"]["nodes"] == 9 and w["c4_n9"]["cfg"]["log_cap"] == 4096
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

