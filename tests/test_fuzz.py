"""Differential fuzzing from random valid states: Python restatement == C oracle (CPU) and
C oracle == GPU kernel (gpu). Each state runs 8 ticks; every field, queue, log and counter must
agree."""
import random

import numpy as np
import pytest

import fuzz
import helpers
import scenarios

TICKS = 8


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_python_equals_oracle(seed):
    rng = random.Random(1000 + seed)
    cfg = fuzz.random_config(rng)
    for _ in range(6):
        scn = fuzz.random_scenario(rng, cfg)
        py = scenarios.run(scn, "py")
        be = scenarios.run(scn, "oracle", helpers.oracle)
        py.step(TICKS)
        be.step(TICKS)
        if be.be.counters()["payload_evicted"]:
            continue
        helpers.compare_py_backend(py.pc, be.be, 0)
        c = be.be.counters()
        for k, v in py.pc.cnt.items():
            assert c[k] == v, (k, c[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(24))
def test_fuzz_gpu_equals_oracle(seed):
    rng = random.Random(5000 + seed)
    cfg = fuzz.random_config(rng)
    scns = [fuzz.random_scenario(rng, cfg) for _ in range(200)]
    g = fuzz.load_batch(helpers.gpu, cfg, scns)
    r = fuzz.load_batch(helpers.oracle, cfg, scns)
    assert np.array_equal(g.digest(), r.digest()), "state load differs"
    for _ in range(TICKS):
        g.step(1)
        r.step(1)
        dg, dr = g.digest(), r.digest()
        bad = np.nonzero(dg != dr)[0]
        assert not len(bad), (f"tick {g.tick - 1}: {len(bad)} clusters differ; first {bad[0]}\n"
                              + helpers.describe_cluster_diff(g, r, int(bad[0])))
    assert g.counters() == r.counters()


def _gpu_vs_oracle_multi_tick(cfg, scns, steps):
    g = fuzz.load_batch(helpers.gpu, cfg, scns)
    r = fuzz.load_batch(helpers.oracle, cfg, scns)
    for n in steps:
        g.step(n)
        r.step(n)
        dg, dr = g.digest(), r.digest()
        bad = np.nonzero(dg != dr)[0]
        assert not len(bad), (f"after tick {g.tick}: {len(bad)} clusters differ; first {bad[0]}\n"
                              + helpers.describe_cluster_diff(g, r, int(bad[0])))
    assert g.counters() == r.counters()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_fuzz_gpu_multi_tick_launch(seed):
    """The same random states stepped several ticks per launch: idle-tick skipping and the
    append-response drain (which need a launch longer than one tick) against the oracle."""
    rng = random.Random(7000 + seed)
    cfg = fuzz.random_config(rng)
    scns = [fuzz.random_scenario(rng, cfg) for _ in range(200)]
    _gpu_vs_oracle_multi_tick(cfg, scns, [8, 5, 40])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_fuzz_gpu_drain(seed):
    """Configurations where the append-response drain runs (faithful model, N <= 5, no client
    traffic, no trace rings), random states with queued responses, short timers (hb 1..6, so a
    leader's heartbeat falls inside a drain), with and without faults."""
    rng = random.Random(9000 + seed)
    cfg = fuzz.random_config(rng)
    cfg.update(nodes=rng.randint(2, 5), variant_flags=rng.choice([0, 1]), client_ppm=0,
               trace_cap=0, trace_entry_cap=0)
    scns = [fuzz.random_scenario(rng, cfg) for _ in range(200)]
    _gpu_vs_oracle_multi_tick(cfg, scns, [8, 8, 64, 200])


def _no_client_sets(scn):
    """Drop queued client-sets: a host-written client-set turns the LITE kernel off."""
    scn.queues = {q: [m for m in ms if m["type"] != "client-set"] for q, ms in scn.queues.items()}
    scn.queues = {q: ms for q, ms in scn.queues.items() if ms}
    return scn


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_fuzz_gpu_lite_queues(seed):
    """LITE configurations (no client traffic, no faults, a fixed delay, N <= 5), where the tick
    kernel keeps each launch's messages in LDS-resident queues: random states whose queued
    messages start the launch in HBM mode, short timers and fixed delays up to 6 ticks (a sender
    then finds its previous message still held: overflow cell + spill), tiny inboxes (LDS-mode
    overflow drops), halted receivers; single-tick and long launches against the oracle."""
    rng = random.Random(11000 + seed)
    cfg = fuzz.random_config(rng)
    d = rng.choice([1, 1, 2, 3, 6])
    cfg.update(nodes=rng.randint(2, 5), client_ppm=0, drop_ppm=0, dup_ppm=0, part_ppm=0,
               dmin=d, dmax=d, trace_cap=0, trace_entry_cap=0,
               inbox_cap=rng.choice([1, 2, 3, 16]), variant_flags=rng.choice([0, 0, 1]))
    scns = [_no_client_sets(fuzz.random_scenario(rng, cfg)) for _ in range(200)]
    _gpu_vs_oracle_multi_tick(cfg, scns, [1, 3, 8, 64, 200, 2000])
