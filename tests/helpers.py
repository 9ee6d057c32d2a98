"""Shared test helpers: oracle handles and state comparison (test infrastructure)."""
from __future__ import annotations

import os
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
ORACLE_LIB = ROOT / "oracle" / "build" / "libraftref.so"

from raftsim._backend import Backend, RaftSimError  # noqa: E402,F401
import pyref  # noqa: E402


def oracle(**cfg):
    return Backend(ORACLE_LIB, "raft_ref_", **cfg)


def py_config(**cfg):
    """pyref config from raft_sim_config_t-style keywords."""
    keys = pyref.default_config().keys()
    return pyref.default_config(**{k: v for k, v in cfg.items() if k in keys})


NODE_FIELDS = ["role", "voted_for", "leader_id", "fault", "entries_is_seq", "ls_present",
               "votes", "ls_keys", "current_term", "commit_index", "log_len", "deadline",
               "next_index", "match_index", "last_led_term", "trace_hash", "req_count",
               "res_count", "commit_count"]


def compare_py_backend(pc: "pyref.PyCluster", be: Backend, cluster: int):
    """Assert a pyref cluster and cluster `cluster` of a backend hold the same logical state."""
    recs = be.read_nodes(cluster, 1)
    for i in range(1, pc.N + 1):
        want = pc.canonical_node(i)
        got = recs[i - 1]
        for f in NODE_FIELDS:
            assert got[f] == want[f], (f"node {i} field {f}: backend {got[f]} != py {want[f]}",
                                       got, want)
        assert be.log(cluster, i) == [tuple(e) for e in pc.logs[i].entries], f"node {i} log"
        cap = be.config.commit_stream_cap
        if cap:
            want_s = pc.stream[i][len(pc.stream[i]) - min(cap, len(pc.stream[i])):]
            assert be.commit_stream(cluster, i) == want_s, f"node {i} commit stream"
        for which in (0, 1):
            gq = be.read_queue(cluster, i, which)
            wq = pc.canonical_msgs(i, which)
            assert len(gq) == len(wq), f"node {i} queue {which} length"
            for g, w in zip(gq, wq):
                assert g[:7] == w[:7], (f"node {i} queue {which}", g, w)
                pcnt = g[1] >> 16
                if pcnt:
                    src = (g[1] >> 3) & 15
                    ar = be.read_arena(cluster, src)
                    A = len(ar)
                    assert [ar[(g[7] + k) % A] for k in range(pcnt)] == [tuple(e) for e in w[7]]
    assert be.read_clusters(cluster, 1)[0] == pc.canonical_cluster()
    if be.config.trace_cap:
        compare_trace(pc, be, cluster)


def compare_trace(pc, be, cluster):
    """F3: the backend's recorded wait events (and their printed form) equal pyref's."""
    for i in range(1, pc.N + 1):
        evs = pc.events[i]
        first = max(0, len(evs) - be.config.trace_cap)
        got = be.trace(cluster, i)
        assert [e["seq"] for e in got] == list(range(first, len(evs))), f"node {i} trace seqs"
        for e, (t, node, msg) in zip(got, evs[first:]):
            assert e["tick"] == t, f"node {i} event {e['seq']} tick"
            want = pyref.encode_msg(0, msg) if msg is not None else None
            if want is None:
                assert e["msg"]["hdr"] == 0 and e["msg"]["arrival"] == 0
            else:
                assert (e["msg"]["hdr"], e["msg"]["term"], e["msg"]["a"], e["msg"]["b"],
                        e["msg"]["eterm"], e["msg"]["eval"]) == want[1:7], (i, e, msg)
        got_txt, want_txt = be.edn_trace(cluster, i), pyref.stdout_of(pc, i, first)
        if "#raft.sim/unretained" in got_txt:    # entries older than the trace-entry ring
            want_txt = "\n".join(
                re.sub(r":entries \[[^\]]*\]", lambda m: f":entries {unretained.pop(0)}", w)
                if (unretained := re.findall(r"#raft.sim/unretained \d+", g)) else w
                for g, w in zip(got_txt.split("\n"), want_txt.split("\n")))
        assert got_txt == want_txt, f"node {i} EDN dump"


def gpu(**cfg):
    import raftsim
    return raftsim.Simulator(**cfg)


def oracle_threads(be, n):
    be._lib.raft_ref_set_threads(be._h, n)


def oracle_idle_skip(be, on=True):
    be._lib.raft_ref_set_idle_skip(be._h, int(on))


def cpu_threads():
    """The host CPUs this process may use: its affinity mask, capped by the cgroup CPU quota (the
    GPU box's share: its affinity mask shows every CPU of the machine, the quota 16 of them)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def describe_cluster_diff(a, b, cluster):
    """Human-readable differences between cluster `cluster` of two backends."""
    lines = []
    ra, rb = a.read_nodes(cluster, 1), b.read_nodes(cluster, 1)
    for i, (x, y) in enumerate(zip(ra, rb)):
        for f in x:
            if x[f] != y[f]:
                lines.append(f"  node {i + 1} {f}: {x[f]} != {y[f]}")
        for which in (0, 1):
            qa, qb = a.read_queue(cluster, i + 1, which), b.read_queue(cluster, i + 1, which)
            if qa != qb:
                lines.append(f"  node {i + 1} queue {which}: {qa} != {qb}")
        la, lb = a.log(cluster, i + 1), b.log(cluster, i + 1)
        if la != lb:
            lines.append(f"  node {i + 1} log: {la[:12]}... != {lb[:12]}...")
    ha, hb = a.read_clusters(cluster, 1), b.read_clusters(cluster, 1)
    if ha != hb:
        lines.append(f"  cluster record {ha} != {hb}")
    return "\n".join(lines)


def bisect_divergence(cfg, g, max_ticks, make_a, make_b):
    """Re-run global cluster g alone, one tick at a time, and report the first divergent tick."""
    one = dict(cfg, n_clusters=1, cluster_offset=g)
    a, b = make_a(**one), make_b(**one)
    prev = None
    for t in range(max_ticks):
        a.step(1)
        b.step(1)
        if a.digest()[0] != b.digest()[0]:
            return (f"cluster {g} first diverges at tick {t}:\n"
                    + describe_cluster_diff(a, b, 0)
                    + (f"\n  state before tick {t} (a):\n{prev}" if prev else ""))
        prev = "\n".join(f"    {r}" for r in a.read_nodes(0, 1)) if t % 1 == 0 else prev
    return f"cluster {g}: no divergence in {max_ticks} single-tick steps (launch-size effect?)"
