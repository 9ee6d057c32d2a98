"""ctypes mirror of include/raftsim.h (the C ABI of libraftsim.so).

The structure layouts here must match the header byte for byte; tests/test_abi.py checks the sizes
and offsets against the C compiler's view.
"""
from __future__ import annotations

import ctypes as C

MAX_NODES = 9
MAX_INBOX = 16

COUNTER_NAMES = ["ev_rv", "ev_ae", "ev_cs", "ev_vr", "ev_ar", "ev_timeout", "ev_heartbeat",
                 "leaders", "sent", "delivered", "dropped", "partitioned", "duplicated",
                 "overflow", "to_halted", "client_injected", "halt_ioobe", "halt_npe", "halt_cce",
                 "halt_overflow", "entries_appended", "entries_applied", "payload_evicted",
                 "viol_election", "viol_log", "viol_complete", "redirects", "client_abandoned"]


class Config(C.Structure):
    _fields_ = [("n_clusters", C.c_uint32), ("cluster_offset", C.c_uint32),
                ("nodes", C.c_uint32), ("log_cap", C.c_uint32), ("arena_cap", C.c_uint32),
                ("inbox_cap", C.c_uint32), ("seed", C.c_uint64), ("hb", C.c_uint32),
                ("el_base", C.c_uint32), ("el_span", C.c_uint32), ("drop_ppm", C.c_uint32),
                ("dup_ppm", C.c_uint32), ("dmin", C.c_uint32), ("dmax", C.c_uint32),
                ("part_ppm", C.c_uint32), ("part_epoch", C.c_uint32),
                ("client_ppm", C.c_uint32), ("variant_flags", C.c_uint32),
                ("device", C.c_int32), ("ticks_per_launch", C.c_uint32),
                ("commit_stream_cap", C.c_uint32), ("trace_cap", C.c_uint32),
                ("trace_entry_cap", C.c_uint32), ("schedule", C.c_uint32),
                ("client_period", C.c_uint32), ("client_burst", C.c_uint32),
                ("client_redirects", C.c_uint32), ("n_devices", C.c_int32)]


class Node(C.Structure):
    _fields_ = [("role", C.c_uint8), ("voted_for", C.c_uint8), ("leader_id", C.c_uint8),
                ("fault", C.c_uint8), ("entries_is_seq", C.c_uint8), ("ls_present", C.c_uint8),
                ("votes", C.c_uint16), ("ls_keys", C.c_uint16), ("reserved0", C.c_uint16),
                ("current_term", C.c_uint32), ("commit_index", C.c_uint32),
                ("log_len", C.c_uint32), ("deadline", C.c_uint32),
                ("next_index", C.c_int32 * MAX_NODES), ("match_index", C.c_int32 * MAX_NODES),
                ("last_led_term", C.c_uint32), ("arena_base", C.c_uint32),
                ("arena_frontier", C.c_uint32), ("req_count", C.c_uint32),
                ("res_count", C.c_uint32), ("commit_count", C.c_uint32),
                ("trace_hash", C.c_uint64)]

    def as_dict(self, n_nodes):
        d = {f: getattr(self, f) for f, _ in self._fields_
             if not f.startswith("reserved")}
        d["next_index"] = list(self.next_index)[:n_nodes]
        d["match_index"] = list(self.match_index)[:n_nodes]
        return d


class Msg(C.Structure):
    _fields_ = [(f, C.c_uint32) for f in
                ("arrival", "hdr", "term", "a", "b", "eterm", "eval", "poff")]

    def words(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class Entry(C.Structure):
    _fields_ = [("term", C.c_uint32), ("val", C.c_uint32)]


class TraceEvent(C.Structure):
    _fields_ = [("tick", C.c_uint32), ("seq", C.c_uint32), ("msg", Msg),
                ("role", C.c_uint8), ("voted_for", C.c_uint8), ("leader_id", C.c_uint8),
                ("ls_present", C.c_uint8), ("votes", C.c_uint16), ("ls_keys", C.c_uint16),
                ("current_term", C.c_uint32), ("next_index", C.c_int32 * MAX_NODES),
                ("match_index", C.c_int32 * MAX_NODES), ("entries_seq", C.c_uint32)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["msg"] = {f: getattr(self.msg, f) for f, _ in Msg._fields_}
        d["next_index"] = list(self.next_index)
        d["match_index"] = list(self.match_index)
        return d


class Cluster(C.Structure):
    _fields_ = [("hwm_index", C.c_uint32), ("hwm_term", C.c_uint32), ("hwm_val", C.c_uint32),
                ("client_next", C.c_uint32), ("client_count", C.c_uint32),
                ("reserved", C.c_uint32 * 3)]

    def as_dict(self):
        return {"hwm": (self.hwm_index, self.hwm_term, self.hwm_val),
                "client_next": self.client_next, "client_count": self.client_count}


class Counters(C.Structure):
    _fields_ = [("node_ticks", C.c_uint64), ("first_violation_tick", C.c_uint64),
                ("c", C.c_uint64 * len(COUNTER_NAMES)), ("payload_max", C.c_uint64)]

    def as_dict(self):
        d = {name: self.c[i] for i, name in enumerate(COUNTER_NAMES)}
        d["node_ticks"] = self.node_ticks
        d["payload_max"] = self.payload_max
        d["first_violation_tick"] = (None if self.first_violation_tick == 2 ** 64 - 1
                                     else self.first_violation_tick)
        return d


P = C.POINTER
_SIGS = {
    "abi_version": (C.c_int, []),
    "default_config": (None, [P(Config)]),
    "create": (C.c_int, [P(Config), P(C.c_void_p)]),
    "step": (C.c_int, [C.c_void_p, C.c_uint32]),
    "step_async": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sync": (C.c_int, [C.c_void_p]),
    "tick": (C.c_uint64, [C.c_void_p]),
    "set_tick": (C.c_int, [C.c_void_p, C.c_uint64]),
    "read_nodes": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Node)]),
    "write_nodes": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Node)]),
    "read_queue": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(Msg),
                             C.c_uint32]),
    "write_queue": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(Msg),
                              C.c_uint32]),
    "read_arena": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Entry), C.c_uint32]),
    "write_arena": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Entry), C.c_uint32]),
    "read_commit_stream": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint32),
                                     C.c_uint32]),
    "write_commit_stream": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint32),
                                      C.c_uint32]),
    "read_trace": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(TraceEvent),
                             C.c_uint32]),
    "read_trace_entries": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(Entry),
                                     C.c_uint32]),
    "read_clusters": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Cluster)]),
    "write_clusters": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(Cluster)]),
    "read_counters": (C.c_int, [C.c_void_p, P(Counters)]),
    "digest": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint64)]),
    "last_step_timing": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_uint32)]),
    "last_span": (C.c_int, [C.c_void_p, P(C.c_double)]),
    "destroy": (None, [C.c_void_p]),
    "last_error": (C.c_char_p, []),
}

# Every symbol include/raftsim.h declares (tests/test_abi.py checks the header agrees).
PRODUCT_SYMBOLS = ["raft_sim_" + n for n in _SIGS]


def bind(lib, prefix, optional=()):
    """Attach argtypes/restype to `lib`'s `prefix + name` functions; return {name: fn}."""
    fns = {}
    for name, (res, args) in _SIGS.items():
        sym = prefix + name
        if not hasattr(lib, sym):
            if name in optional:
                continue
            raise OSError(f"{sym} missing from {lib._name}")
        f = getattr(lib, sym)
        f.restype = res
        f.argtypes = args
        fns[name] = f
    return fns
