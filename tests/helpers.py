"""Shared test helpers: oracle handles and state comparison (test infrastructure)."""
from __future__ import annotations

from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
ORACLE_LIB = ROOT / "oracle" / "build" / "libraftref.so"

from raftsim._backend import Backend  # noqa: E402
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
               "res_count"]


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
    assert be.read_hwm(cluster, 1)[0] == tuple(pc.hwm)
