"""Host-side handle over a library that implements the include/raftsim.h ABI."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi

ROLE_NAMES = {0: ":follower", 1: ":candidate", 2: ":leader", 3: ":follwer"}
FAULT_NAMES = {0: None, 1: "IndexOutOfBoundsException", 2: "NullPointerException",
               3: "ClassCastException", 4: "LogCapacityExceeded"}


class RaftSimError(RuntimeError):
    pass


def make_config(fns, **kw) -> _abi.Config:
    cfg = _abi.Config()
    fns["default_config"](C.byref(cfg))
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown config field {k!r}")
        setattr(cfg, k, v)
    return cfg


class Backend:
    """One simulator handle. `lib_path` + `prefix` select the implementation."""

    def __init__(self, lib_path, prefix, **config):
        self._lib = C.CDLL(str(lib_path))
        self._fns = _abi.bind(self._lib, prefix, optional=("last_step_timing", "last_span"))
        if self._fns["abi_version"]() != 2:
            raise RaftSimError("ABI version mismatch")
        self.config = make_config(self._fns, **config)
        h = C.c_void_p()
        self._check(self._fns["create"](C.byref(self.config), C.byref(h)))
        self._h = h
        self.N = self.config.nodes
        self.C = self.config.n_clusters

    # -- plumbing -------------------------------------------------------------------------------
    def _check(self, rc):
        if rc < 0:
            raise RaftSimError(f"rc={rc}: {self._fns['last_error']().decode()}")
        return rc

    def close(self):
        if getattr(self, "_h", None):
            self._fns["destroy"](self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- stepping -------------------------------------------------------------------------------
    def step(self, n_ticks):
        self._check(self._fns["step"](self._h, int(n_ticks)))

    def step_async(self, n_ticks):
        """Enqueue n_ticks without waiting (the oracle runs them at once); see sync()."""
        self._check(self._fns["step_async"](self._h, int(n_ticks)))

    def sync(self):
        self._check(self._fns["sync"](self._h))

    @property
    def tick(self):
        return int(self._fns["tick"](self._h))

    def set_tick(self, tick):
        """Resume at `tick` (state restored through the write_* calls; SIM_SPEC deadlines are
        absolute ticks)."""
        self._check(self._fns["set_tick"](self._h, int(tick)))

    def last_step_timing(self):
        ms, n = C.c_double(), C.c_uint32()
        self._check(self._fns["last_step_timing"](self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def last_span(self):
        """Device ms of everything the last step (or the steps since the previous sync) enqueued."""
        ms = C.c_double()
        self._check(self._fns["last_span"](self._h, C.byref(ms)))
        return ms.value

    # -- state ----------------------------------------------------------------------------------
    def read_nodes_raw(self, c0=0, nc=None):
        nc = self.C - c0 if nc is None else nc
        arr = (_abi.Node * (nc * self.N))()
        self._check(self._fns["read_nodes"](self._h, c0, nc, arr))
        return arr

    def read_nodes(self, c0=0, nc=None):
        return [n.as_dict(self.N) for n in self.read_nodes_raw(c0, nc)]

    def write_nodes(self, c0, records):
        nc = len(records) // self.N
        arr = (_abi.Node * len(records))()
        for i, r in enumerate(records):
            if isinstance(r, _abi.Node):
                arr[i] = r
                continue
            for k, v in r.items():
                if k in ("next_index", "match_index"):
                    getattr(arr[i], k)[:len(v)] = list(v)
                elif k not in ("req_count", "res_count"):
                    setattr(arr[i], k, v)
        self._check(self._fns["write_nodes"](self._h, c0, nc, arr))

    def read_queue(self, cluster, node_id, which):
        buf = (_abi.Msg * _abi.MAX_INBOX)()
        n = self._check(self._fns["read_queue"](self._h, cluster, node_id, which, buf,
                                                _abi.MAX_INBOX))
        return [buf[i].words() for i in range(n)]

    def write_queue(self, cluster, node_id, which, msgs):
        buf = (_abi.Msg * max(1, len(msgs)))()
        for i, w in enumerate(msgs):
            for f, v in zip(("arrival", "hdr", "term", "a", "b", "eterm", "eval", "poff"), w):
                setattr(buf[i], f, v)
        self._check(self._fns["write_queue"](self._h, cluster, node_id, which, buf, len(msgs)))

    def read_arena(self, cluster, node_id):
        A = self._check(self._fns["read_arena"](self._h, cluster, node_id, None, 0))
        buf = (_abi.Entry * A)()
        self._check(self._fns["read_arena"](self._h, cluster, node_id, buf, A))
        return [(e.term, e.val) for e in buf]

    def write_arena(self, cluster, node_id, entries):
        buf = (_abi.Entry * max(1, len(entries)))()
        for i, (t, v) in enumerate(entries):
            buf[i].term, buf[i].val = t, v
        self._check(self._fns["write_arena"](self._h, cluster, node_id, buf, len(entries)))

    def log(self, cluster, node_id):
        """The node's logical log :entries (log.clj:33-34) as (term, val) tuples."""
        rec = self.read_nodes(cluster, 1)[node_id - 1]
        ar = self.read_arena(cluster, node_id)
        A = len(ar)
        return [ar[(rec["arena_base"] + i) % A] for i in range(rec["log_len"])]

    def commit_stream(self, cluster, node_id):
        """F2: the committed :val's apply-entries! wrote to node_<id>.log (log.clj:69-76), as far
        back as the configured ring (commit_stream_cap) reaches, oldest first."""
        cap = max(1, self.config.commit_stream_cap)
        buf = (C.c_uint32 * cap)()
        n = self._check(self._fns["read_commit_stream"](self._h, cluster, node_id, buf, cap))
        return list(buf[:n])

    def write_commit_stream(self, cluster, node_id, vals):
        buf = (C.c_uint32 * max(1, len(vals)))(*vals)
        self._check(self._fns["write_commit_stream"](self._h, cluster, node_id, buf, len(vals)))

    def write_commit_logs(self, directory, cluster=0):
        """Write node_<id>.log files the way the reference's Log component does (log.clj:16-18):
        one committed value per line. Only the retained tail of the stream is available."""
        from pathlib import Path
        d = Path(directory)
        d.mkdir(parents=True, exist_ok=True)
        for i in range(1, self.N + 1):
            (d / f"node_{i}.log").write_text("".join(f"{v}\n" for v in self.commit_stream(cluster, i)))

    def trace(self, cluster, node_id, first=0):
        """F3: the node's recorded `wait` iterations with seq >= first (core.clj:182-186), oldest
        first, as dicts of raft_trace_event_t fields."""
        out, cap = [], max(1, self.config.trace_cap)
        buf = (_abi.TraceEvent * cap)()
        while True:
            n = self._check(self._fns["read_trace"](self._h, cluster, node_id, first, buf, cap))
            out.extend(buf[i].as_dict() for i in range(n))
            if n < cap:
                return out
            first = out[-1]["seq"] + 1

    def trace_entries(self, cluster, node_id, first, count):
        """The `count` trace-entry-ring entries from index `first` as (term, val) pairs, or None
        when the ring no longer holds them all (or trace_entry_cap is 0)."""
        buf = (_abi.Entry * max(1, count))()
        n = self._fns["read_trace_entries"](self._h, cluster, node_id, first, buf, count)
        if n != count:
            return None
        return [(buf[i].term, buf[i].val) for i in range(n)]

    def edn_trace(self, cluster, node_id, first=0, set_order="sorted"):
        """The reference's stdout for node `node_id` of `cluster` from event `first` on:
        `; Node` / (prn node) / `; Message` / (prn message) per wait (core.clj:182-186)."""
        from . import edn
        parts = []
        for e in self.trace(cluster, node_id, first):
            entries = None
            if (e["msg"]["hdr"] & 7) == 2:
                cnt = e["msg"]["hdr"] >> 16
                entries = self.trace_entries(cluster, node_id, e["entries_seq"], cnt) if cnt else []
            parts.append(edn.format_event(e, entries, node_id, self.N, set_order))
        return "".join(parts)

    def write_traces(self, directory, cluster=0, set_order="sorted"):
        """One file per node, node_<id>.out, holding what that node's JVM prints per event."""
        from pathlib import Path
        d = Path(directory)
        d.mkdir(parents=True, exist_ok=True)
        for i in range(1, self.N + 1):
            (d / f"node_{i}.out").write_text(self.edn_trace(cluster, i, set_order=set_order))

    def read_clusters(self, c0=0, nc=None):
        """Per-cluster records: checker high-water mark and client-injection cursor."""
        nc = self.C - c0 if nc is None else nc
        arr = (_abi.Cluster * nc)()
        self._check(self._fns["read_clusters"](self._h, c0, nc, arr))
        return [r.as_dict() for r in arr]

    def write_clusters(self, c0, recs):
        arr = (_abi.Cluster * len(recs))()
        for i, r in enumerate(recs):
            arr[i].hwm_index, arr[i].hwm_term, arr[i].hwm_val = r["hwm"]
            arr[i].client_next, arr[i].client_count = r["client_next"], r["client_count"]
        self._check(self._fns["write_clusters"](self._h, c0, len(recs), arr))

    def counters(self):
        c = _abi.Counters()
        self._check(self._fns["read_counters"](self._h, C.byref(c)))
        return c.as_dict()

    def digest(self, c0=0, nc=None):
        nc = self.C - c0 if nc is None else nc
        out = np.zeros(nc, dtype=np.uint64)
        self._check(self._fns["digest"](self._h, c0, nc,
                                        out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    # -- reference vocabulary -------------------------------------------------------------------
    def node_map(self, cluster, node_id):
        """The node as the reference's `prn node` would show it (core.clj:31-38,182-183)."""
        r = self.read_nodes(cluster, 1)[node_id - 1]
        ls = None
        if r["ls_present"]:
            keys = [p for p in range(1, self.N + 1) if (r["ls_keys"] >> p) & 1]
            ls = {":next-index": {p: r["next_index"][p - 1] for p in keys},
                  ":match-index": {p: r["match_index"][p - 1] for p in keys}}
        return {":id": node_id, ":state": ROLE_NAMES[r["role"]],
                ":current-term": r["current_term"],
                ":voted-for": r["voted_for"] or None, ":leader-id": r["leader_id"] or None,
                ":leader-state": ls,
                ":votes": {p for p in range(1, self.N + 1) if (r["votes"] >> p) & 1},
                "halted": FAULT_NAMES[r["fault"]]}
