"""The C oracle against the Python restatement (random configs) and the Philox KAT."""
import ctypes
import random

import pytest

import helpers
import pyref

KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD))]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_kat_python(ctr, key, want):
    assert pyref.philox(ctr, key) == want


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_kat_c(ctr, key, want):
    lib = ctypes.CDLL(str(helpers.ORACLE_LIB))
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib.raft_ref_philox(c, k, o)
    assert tuple(o) == want


def random_config(rng):
    n = rng.choice([2, 3, 4, 5, 5, 5, 6, 7, 8, 9])
    cfg = dict(nodes=n, seed=rng.getrandbits(64), log_cap=rng.choice([8, 32, 128]),
               inbox_cap=rng.choice([1, 2, 4, 16]))
    if rng.random() < 0.7:
        dmin = rng.randint(1, 5)
        cfg.update(drop_ppm=rng.choice([0, 50000, 200000]), dup_ppm=rng.choice([0, 20000, 300000]),
                   dmin=dmin, dmax=dmin + rng.randint(0, 40))
    if rng.random() < 0.5:
        cfg.update(part_ppm=rng.choice([50000, 300000]), part_epoch=rng.choice([100, 1000]))
    cfg["client_ppm"] = rng.choice([0, 100, 1000, 20000])
    if cfg["client_ppm"] and rng.random() < 0.6:       # bursts + followed redirects (D14, D15)
        cfg["client_redirects"] = rng.choice([0, 1, 2, 4, 16])
        if rng.random() < 0.7:
            period = rng.choice([7, 300, 2000, 16384])
            cfg.update(client_period=period, client_burst=rng.randint(1, period),
                       client_ppm=rng.choice([20000, 200000, 1000000]))
    if rng.random() < 0.5:
        cfg.update(hb=rng.randint(5, 300), el_base=rng.randint(5, 500), el_span=rng.randint(1, 500))
    if rng.random() < 0.2:
        cfg["variant_flags"] = 1
    if rng.random() < 0.3:
        cfg["arena_cap"] = 2 * cfg["log_cap"]
    cfg["commit_stream_cap"] = rng.choice([0, 3, 64])
    cfg["trace_cap"] = rng.choice([0, 3, 4096])
    cfg["trace_entry_cap"] = 1 << 16 if cfg["trace_cap"] else 0
    return cfg


@pytest.mark.parametrize("seed", range(24))
def test_oracle_equals_python_restatement(seed):
    rng = random.Random(seed)
    cfg = random_config(rng)
    gid = rng.randrange(1 << 20)
    ticks = 6000
    be = helpers.oracle(n_clusters=1, cluster_offset=gid, **cfg)
    pc = pyref.PyCluster(helpers.py_config(**cfg), gid)
    for chunk in range(3):
        for t in range(chunk * ticks // 3, (chunk + 1) * ticks // 3):
            pc.step(t)
        be.step(ticks // 3)
        c = be.counters()
        if c["payload_evicted"]:
            pytest.skip("arena eviction: the Python restatement models ideal snapshots")
        helpers.compare_py_backend(pc, be, 0)
    c = be.counters()
    for k, v in pc.cnt.items():
        assert c[k] == v, (k, c[k], v)
    assert c["first_violation_tick"] == pc.first_violation


@pytest.mark.parametrize("seed", range(24))
def test_spec_oracle_equals_python_restatement(seed):
    """F4 Spec-Raft (flag 2) and its bug-injected form (flags 3), same cross-check."""
    rng = random.Random(7000 + seed)
    cfg = random_config(rng)
    cfg["variant_flags"] = rng.choice([2, 3])
    gid = rng.randrange(1 << 20)
    be = helpers.oracle(n_clusters=1, cluster_offset=gid, **cfg)
    pc = pyref.PyCluster(helpers.py_config(**cfg), gid)
    for t in range(6000):
        pc.step(t)
    be.step(6000)
    c = be.counters()
    if c["payload_evicted"]:
        pytest.skip("arena eviction: the Python restatement models ideal snapshots")
    helpers.compare_py_backend(pc, be, 0)
    for k, v in pc.cnt.items():
        assert c[k] == v, (k, c[k], v)
    assert c["first_violation_tick"] == pc.first_violation


FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)


@pytest.mark.parametrize("nodes", [3, 4, 5, 7])
def test_spec_raft_is_safe_and_the_injected_bug_is_not(nodes):
    """BASELINE config 5 on the CPU: the Spec-Raft control (SIM_SPEC §8) shows no violation of
    election safety, log matching or leader completeness under drop/dup/delay/partitions with
    client traffic and fast timers, while dropping only the up-to-date vote check (flags 3) lets a
    stale candidate win and lose committed entries (leader completeness)."""
    base = dict(n_clusters=512, nodes=nodes, seed=5, client_ppm=10000, log_cap=512, hb=300,
                el_base=500, el_span=500, **FAULTS)
    ctl = helpers.oracle(variant_flags=2, **base)
    bug = helpers.oracle(variant_flags=3, **base)
    for be in (ctl, bug):
        helpers.oracle_threads(be, helpers.cpu_threads())
        be.step(30000)
    c, b = ctl.counters(), bug.counters()
    assert c["leaders"] > 1000 and c["entries_applied"] > 10000
    assert c["viol_election"] == c["viol_log"] == c["viol_complete"] == 0
    assert c["first_violation_tick"] is None
    assert b["viol_complete"] > 0 and b["viol_election"] == 0
    assert b["first_violation_tick"] is not None


@pytest.mark.parametrize("redirects", [0, 3])
def test_message_conservation(redirects):
    """sent + client_injected + redirects - dropped - partitioned + duplicated
    = delivered + overflow + to_halted; every client-set a non-leader handles is either
    re-sent along the redirect (redirects) or abandoned."""
    be = helpers.oracle(n_clusters=64, nodes=5, seed=5, drop_ppm=100000, dup_ppm=50000, dmax=20,
                        part_ppm=100000, client_ppm=20000, inbox_cap=3, log_cap=64,
                        client_period=4000, client_burst=800, client_redirects=redirects)
    be.step(20000)
    c = be.counters()
    assert (c["sent"] + c["client_injected"] + c["redirects"] - c["dropped"] - c["partitioned"]
            + c["duplicated"] == c["delivered"] + c["overflow"] + c["to_halted"])
    assert c["redirects"] > 0 if redirects else c["redirects"] == 0
    assert c["client_abandoned"] > 0


def test_client_schedule_bursts():
    """D14: client-sets arrive only in the first client_burst ticks of every client_period."""
    import pyref
    P, B = 1000, 150
    for j in range(0, 5000, 7):
        t = pyref.on_tick(j, P, B)
        assert t % P < B and pyref.on_index(t, P, B) == j
    be = helpers.oracle(n_clusters=32, nodes=5, seed=3, client_ppm=300000, client_period=P,
                        client_burst=B, trace_cap=4096)
    be.step(6000)
    ticks = [e["tick"] for c in range(32) for i in range(1, 6) for e in be.trace(c, i)
             if (e["msg"]["hdr"] & 7) == 3 and e["msg"]["arrival"] == e["tick"]]
    assert ticks and all(t % P < B for t in ticks)
    assert be.counters()["client_injected"] > 0.2 * 32 * 6 * B


def test_commit_logs_written_like_the_reference(tmp_path):
    """F2: node_<id>.log holds one committed :val per line (log.clj:16-18)."""
    be = helpers.oracle(n_clusters=4, nodes=5, seed=7, client_ppm=3000, log_cap=256,
                        commit_stream_cap=4096)
    be.step(30000)
    be.write_commit_logs(tmp_path, cluster=2)
    for i in range(1, 6):
        lines = (tmp_path / f"node_{i}.log").read_text().splitlines()
        assert [int(x) for x in lines] == be.commit_stream(2, i)
        assert len(lines) == be.read_nodes(2, 1)[i - 1]["commit_count"]
    assert be.counters()["entries_applied"] == sum(r["commit_count"] for r in be.read_nodes())


IDLE_CASES = {
    "bursts": dict(n_clusters=61, nodes=5, seed=13, client_ppm=50000, drop_ppm=50000, dmax=30,
                   part_ppm=100000, log_cap=128, client_period=5000, client_burst=700,
                   client_redirects=3, trace_cap=64, trace_entry_cap=512),
    # crash storm: IOOBE/OVERFLOW halts under client traffic, most client-sets reach halted nodes
    "crash_storm": dict(n_clusters=61, nodes=5, seed=13, client_ppm=80000, drop_ppm=100000,
                        dup_ppm=10000, dmax=50, part_ppm=100000, log_cap=16, client_period=16384,
                        client_burst=2048, client_redirects=4, hb=300, el_base=500, el_span=500),
}


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("case", list(IDLE_CASES))
def test_idle_skipping_does_not_change_results(case, variant):
    """The CPU baseline's discrete-event skipping visits only ticks with something due and gives
    the every-tick restatement's results exactly."""
    cfg = dict(IDLE_CASES[case], variant_flags=variant)
    a, b = helpers.oracle(**cfg), helpers.oracle(**cfg)
    helpers.oracle_idle_skip(b)
    for n in (1, 4999, 7000, 3, 9000):
        a.step(n)
        b.step(n)
        assert (a.digest() == b.digest()).all() and a.counters() == b.counters()
    if case == "crash_storm" and variant == 0:
        assert a.counters()["to_halted"] > a.counters()["client_injected"] // 4


def test_threads_do_not_change_results():
    cfg = dict(n_clusters=97, nodes=7, seed=3, client_ppm=1000, drop_ppm=50000, dmax=9)
    a, b = helpers.oracle(**cfg), helpers.oracle(**cfg)
    helpers.oracle_threads(b, 5)
    a.step(7000)
    b.step(7000)
    assert (a.digest() == b.digest()).all() and a.counters() == b.counters()


def test_sharded_oracle_equals_single():
    """n_devices = G splits the clusters into G independent shards (the product's multi-GPU
    handle, include/raftsim.h); every G gives the same clusters, counters and routed reads."""
    cfg = dict(n_clusters=203, nodes=5, seed=71, client_ppm=80000, log_cap=128,
               client_period=3000, client_burst=600, client_redirects=4, **FAULTS)
    one = helpers.oracle(**cfg)
    one.step(9000)
    for g in (2, 3, 8):
        many = helpers.oracle(n_devices=g, **cfg)
        many.step(9000)
        assert (one.digest() == many.digest()).all()
        assert one.counters() == many.counters()
        assert one.read_nodes(60, 90) == many.read_nodes(60, 90)
        assert one.read_clusters(0, 203) == many.read_clusters(0, 203)
        for c in (0, 67, 68, 101, 202):
            assert one.read_queue(c, 2, 0) == many.read_queue(c, 2, 0)
            assert one.log(c, 3) == many.log(c, 3)


def test_resume_and_tick_horizon():
    """set_tick + the write_* calls resume a run exactly (deadlines are absolute ticks); steps
    whose timers could reach 2^32 - 1 are refused (SIM_SPEC D1)."""
    cfg = dict(n_clusters=16, nodes=5, seed=3, client_ppm=3000, log_cap=64, **FAULTS)
    src = helpers.oracle(**cfg)
    src.step(7000)
    dst = helpers.oracle(**cfg)
    dst.set_tick(7000)
    dst.write_nodes(0, src.read_nodes_raw())
    dst.write_clusters(0, src.read_clusters())
    for c in range(16):
        for i in range(1, 6):
            dst.write_arena(c, i, src.read_arena(c, i))
            for w in (0, 1):
                dst.write_queue(c, i, w, src.read_queue(c, i, w))
    for be in (src, dst):
        be.step(5000)
    assert (src.digest() == dst.digest()).all()
    top = 2 ** 32 - 1 - 10000
    src.set_tick(top - 100)
    src.step(99)
    with pytest.raises(helpers.RaftSimError, match="2\\^32"):
        src.step(2)
    with pytest.raises(helpers.RaftSimError):
        src.set_tick(top + 5)


def test_client_gap_without_client_rate():
    """client_ppm = 0 with a host-written cursor (SIM_SPEC §4 P0): that one injection happens, and
    the gap after it is 2^32 - 1 (never), as the exact integer search gives (pw_i = 2^32)."""
    cfg = dict(n_clusters=8, nodes=5, seed=77, client_ppm=0, log_cap=64)
    r = helpers.oracle(**cfg)
    r.write_clusters(0, [dict(hwm=(0, 0, 0), client_next=100 + i, client_count=i)
                         for i in range(8)])
    r.step(5000)
    assert r.counters()["client_injected"] == 8
    assert all(c["client_next"] == 0xFFFFFFFF for c in r.read_clusters())
    assert pyref.client_gap(12345, pyref.client_powers(0)) == 2 ** 32 - 1


def test_trace_words_are_u32_like_the_c_oracle():
    """The trace-hash words take t, msg_term and current_term as uint32, as raftref.c and the
    kernels do (SIM_SPEC §4): a term at or past 2^32 contributes its low 32 bits only."""
    pc = pyref.PyCluster(pyref.default_config(), 0)
    node = dict(pyref.init_node(1), **{"current-term": (1 << 32) + 5})
    msg = {"type": "append-entries", "term": (1 << 33) + 7, "leader-id": 2}
    lo, hi = pc._trace_words((1 << 32) + 9, 2, msg, node, 0)
    assert lo & 0xFFFFFFFF == 9 and hi == 7 | 5 << 32
    assert max(lo, hi) < 1 << 64
