"""GPU parity over the exact windows bench.py times, at the sizes it times them.

Each test takes its configuration, cluster count and tick window from bench.py's WORKLOADS and
argument defaults (the driver runs `bench.py --steps 20 --warmup 5`), steps the GPU the way the
bench does (step_async + sync per step for from-init windows, K steps enqueued back to back for
steady windows), and compares per-cluster digests (SIM_SPEC §6) with the C oracle's literal
restatement of core.clj/log.clj. Philox is keyed by the global cluster id, so a slice of a
1,048,576-cluster run is checkable on its own: the oracle runs the slice alone with its
cluster_offset. Reference: core.clj:56-67,105-123,141-164 (replication, heartbeats, responses),
log.clj:61-81 (entries-from, append-entries!, remove-from!).
"""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

import helpers
from raftsim import dist as rdist

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
TICKS = 10000


def _bench():
    spec = importlib.util.spec_from_file_location("bench_windows", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


BENCH = _bench()
STEPS, WARMUP = 20, 5          # the driver's fixed command; bench.py's defaults (test_bench_contract)


def _oracle(**cfg):
    r = helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    helpers.oracle_idle_skip(r, True)
    return r


def _check_slices(g, cfg, total, part, when):
    """First, middle and last `part` clusters of the GPU handle vs the oracle run alone on each."""
    for lo in (0, (total // 2) - part // 2, total - part):
        r = _oracle(n_clusters=part, cluster_offset=lo, **cfg)
        r.step(when)
        bad = np.nonzero(g.digest(lo, part) != r.digest())[0]
        assert not len(bad), (f"after {when} ticks: {len(bad)} clusters of [{lo}, {lo + part}) "
                              f"differ; first {lo + int(bad[0])}")
        r.close()


def test_gpu_c2_bench_window():
    """C2's window exactly as the driver times it: seed 42, 65,536 clusters, 5 warm-up steps, then
    20 steps enqueued back to back on the steady kernel with no cluster bailed; digest-equal to
    the oracle after the warm-up and at the end, every counter equal."""
    spec = BENCH.WORKLOADS["c2"]
    cfg = dict(n_clusters=spec["clusters"], **spec["cfg"])
    g, r = helpers.gpu(**cfg), _oracle(**cfg)
    for _ in range(WARMUP):
        g.step(TICKS)
    r.step(WARMUP * TICKS)
    assert np.array_equal(g.digest(), r.digest())
    for _ in range(STEPS):
        g.step_async(TICKS)
    g.sync()
    r.step(STEPS * TICKS)
    assert g.diag_last_bails() == 0
    assert np.array_equal(g.digest(), r.digest())
    assert g.counters() == r.counters()


@pytest.mark.parametrize("name", ["c3", "c3_spec"])
def test_gpu_c3_bench_window_sampled(name):
    """C3 / C3-spec over the bench's whole window: 1,048,576 clusters, ticks [0, 200k) from
    init-node, one sync per step as the bench runs it. The first, middle and last 4,096
    clusters are digest-equal to the oracle at 100k ticks and at the window's end -- the late
    crash-storm part (most faithful nodes halted, logs at their cap, 1000+-entry payloads under
    Spec-Raft) included; nothing was evicted anywhere (SIM_SPEC §4 P3)."""
    spec = BENCH.WORKLOADS[name]
    total, part = spec["clusters"], 4096
    g = helpers.gpu(n_clusters=total, **spec["cfg"])
    try:
        for step in range(1, STEPS + 1):
            g.step_async(TICKS)
            g.sync()
            if step == STEPS // 2:
                _check_slices(g, spec["cfg"], total, part, step * TICKS)
        c = g.counters()
        assert c["payload_evicted"] == 0
        assert c["node_ticks"] == total * 5 * STEPS * TICKS and c["client_injected"] > 0
        _check_slices(g, spec["cfg"], total, part, STEPS * TICKS)
    finally:
        g.close()


@pytest.mark.parametrize("name", ["c4_n7", "c4_n9", "c4_spec"])
def test_gpu_c4_bench_window(name):
    """Config 4 over the bench's window: 16,384 seven- / nine-node clusters with 4096-entry logs,
    ticks [0, 200k) from init-node. Replication is inside the window (AppendEntries batches of
    1000+ entries, core.clj:56-67 shipping the whole suffix), and so are the OVERFLOW halts; the
    first, middle and last 2,048 clusters are digest-equal to the oracle at the end."""
    spec = BENCH.WORKLOADS[name]
    total, part = spec["clusters"], 2048
    g = helpers.gpu(n_clusters=total, **spec["cfg"])
    try:
        for _ in range(STEPS):
            g.step_async(TICKS)
            g.sync()
        c = g.counters()
        assert c["payload_evicted"] == 0
        assert c["ev_ae"] > 10 * total and c["payload_max"] >= 1000
        _check_slices(g, spec["cfg"], total, part, STEPS * TICKS)
    finally:
        g.close()


def test_gpu_c5_time_to_violation_bit_exact():
    """Config 5 as bench.py runs it: 131,072 clusters of the no-up-to-date-check Spec-Raft variant,
    stepped 1,000 ticks at a time until a violation is counted; the oracle, stepped the same way
    on the same clusters, stops in the same chunk with the same first-violation tick and equal
    digests of every cluster."""
    spec = BENCH.WORKLOADS["c5"]
    cfg = dict(n_clusters=spec["clusters"], **spec["cfg"])
    g = helpers.gpu(**cfg)
    fv, ticks, _ = rdist.first_violation_search(g, spec["chunk"], spec["max_ticks"])
    assert fv is not None
    r = _oracle(**cfg)
    cfv, cticks, _ = rdist.first_violation_search(r, spec["chunk"], ticks)
    assert (cfv, cticks) == (fv, ticks)
    assert np.array_equal(g.digest(), r.digest())
    assert g.counters() == r.counters()


def test_gpu_bench_line_is_one_parseable_line(tmp_path):
    """bench.py run as the driver runs it (a child process, C2 headline plus one more workload):
    stdout ends with ONE JSON line well under the ~8,000 characters the driver keeps, carrying the
    headline keys, roofline and cpu_baseline; the full records land in --full-json."""
    import json
    import subprocess
    import sys

    full = tmp_path / "full.json"
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1",
                          "--workload", "c2+c4_n9", "--clusters", "4096", "--full-json", str(full)],
                         capture_output=True, text=True, timeout=600, cwd=str(ROOT))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert lines and len(lines[-1]) < 6000, len(lines[-1]) if lines else None
    rec = json.loads(lines[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline",
              "cpu_baseline", "config", "workloads"):
        assert k in rec, k
    assert rec["steps"] == 2 and rec["warmup"] == 1 and rec["value"] > 0
    assert rec["roofline"]["avg_launch_ms"] > 0 and rec["cpu_baseline"]["value"] > 0
    assert set(json.loads(full.read_text())["workloads"]) == {"c2", "c4_n9"}
