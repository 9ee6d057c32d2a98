"""F3: the reference's per-event stdout, rebuilt from recorded trace events.

Every iteration of `wait` prints (src/raft/core.clj:182-186)

    ; Node
    <(prn node): the node map before the handler runs>
    ; Message
    <(prn message): what alts!! returned; nil for a timeout>
    <blank line>

The simulator records each iteration as a raft_trace_event_t (include/raftsim.h, SIM_SPEC §7); this
module renders those records in Clojure 1.6's printed form:

* node maps keep init-node's key order (core.clj:31-38); every handler only `assoc`s existing
  keys, so the order never changes;
* request messages are the JSON body in the sender's literal key order (core.clj:51-54,62-67), then
  `:type` (server.clj:14-16) and `:resp-chan` (server.clj:21); reply bodies keep the responder's
  order `{:term :id :type ...}` with the outcome keys appended (core.clj:94,98-103,109-121);
* entries print as `{:term t, :val v}` (log.clj:67);
* the channel prints as `#<ManyToManyChannel ...@hash>`; its identity hash is not reproducible, so
  the node-local event number stands in for it.

Two orderings cannot be recovered from the canonical state and are documented in SIM_SPEC §7:
`:votes` sets print sorted by default (`set_order="clojure"` reproduces PersistentHashSet's
iteration order from Clojure 1.6's Murmur3 `hasheq` of longs — derived from the published algorithm,
not checked against a JVM), and a partial leader-state built by `assoc-in` on a non-leader
(core.clj:148-149) prints its peers ascending rather than in first-insertion order.
"""
from __future__ import annotations

ROLE_KW = {0: ":follower", 1: ":candidate", 2: ":leader", 3: ":follwer"}
TYPE_KW = {1: ":request-vote", 2: ":append-entries", 3: ":client-set", 4: ":vote-response",
           5: ":append-response"}
CHAN = ("#<ManyToManyChannel clojure.core.async.impl.channels.ManyToManyChannel@{:x}>")


class Raw(str):
    """Text printed verbatim (the channel object, tagged placeholders)."""


# ------------------------------------------------------------------------------------------------
# Clojure 1.6 hash-set iteration order for small integers (optional)
# ------------------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_k1(k):
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl(k, 15)
    return (k * 0x1B873593) & _M32


def _mix_h1(h, k):
    h ^= k
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & _M32


def _fmix(h, length):
    h ^= length
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def murmur3_hash_long(x: int) -> int:
    """clojure.lang.Murmur3.hashLong (the `hasheq` of Integer/Long in Clojure 1.6), unsigned."""
    if x == 0:
        return 0
    x &= 0xFFFFFFFFFFFFFFFF
    h = _mix_h1(0, _mix_k1(x & _M32))
    h = _mix_h1(h, _mix_k1(x >> 32))
    return _fmix(h, 8)


def _hamt_key(x: int):
    """PersistentHashMap visits keys by successive 5-bit hash chunks, low bits first."""
    h = murmur3_hash_long(x)
    return tuple((h >> s) & 31 for s in range(0, 32, 5))


# ------------------------------------------------------------------------------------------------
# printer
# ------------------------------------------------------------------------------------------------
def edn(v, set_order="sorted") -> str:
    """`prn` of the value shapes the node map and messages hold."""
    if v is None:
        return "nil"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, Raw):
        return str(v)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, str):
        return v                       # keywords are stored with their leading colon
    if isinstance(v, dict):
        return "{" + ", ".join(f"{edn(k, set_order)} {edn(x, set_order)}"
                               for k, x in v.items()) + "}"
    if isinstance(v, (set, frozenset)):
        items = sorted(v, key=_hamt_key) if set_order == "clojure" else sorted(v)
        return "#{" + " ".join(edn(x, set_order) for x in items) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(edn(x, set_order) for x in v) + "]"
    raise TypeError(f"no EDN form for {type(v).__name__}")


def node_map(ev: dict, node_id: int, n_nodes: int) -> dict:
    """The node map of init-node's shape (core.clj:31-38) from a decoded trace event."""
    ls = None
    if ev["ls_present"]:
        keys = [p for p in range(1, n_nodes + 1) if (ev["ls_keys"] >> p) & 1]
        ls = {":next-index": {p: ev["next_index"][p - 1] for p in keys},
              ":match-index": {p: ev["match_index"][p - 1] for p in keys}}
    return {":id": node_id, ":state": ROLE_KW[ev["role"]], ":current-term": ev["current_term"],
            ":voted-for": ev["voted_for"] or None, ":leader-id": ev["leader_id"] or None,
            ":leader-state": ls,
            ":votes": {p for p in range(1, n_nodes + 1) if (ev["votes"] >> p) & 1}}


def message_map(ev: dict, entries):
    """The message alts!! returned, or None for a timeout. `entries` are the append-entries'
    :entries as (term, val) pairs, or None when the trace-entry ring no longer holds them."""
    m = ev["msg"]
    hdr = m["hdr"]
    typ = hdr & 7
    if typ == 0:
        return None
    src, flag, ep, pcnt = (hdr >> 3) & 15, (hdr >> 7) & 1, (hdr >> 8) & 1, hdr >> 16
    entry = {":term": m["eterm"], ":val": m["eval"]} if ep else None
    chan = Raw(CHAN.format(ev["seq"]))
    if typ == 1:
        return {":term": m["term"], ":candidate-id": src, ":last-log-index": m["a"],
                ":last-log-term": entry, ":type": TYPE_KW[1], ":resp-chan": chan}
    if typ == 2:
        if entries is None:
            ents = Raw(f"#raft.sim/unretained {pcnt}")
        else:
            ents = [{":term": t, ":val": v} for t, v in entries]
        return {":term": m["term"], ":leader-id": src, ":leader-commit": m["a"],
                ":prev-log-index": m["b"], ":prev-log-term": entry, ":entries": ents,
                ":type": TYPE_KW[2], ":resp-chan": chan}
    if typ == 3:
        return {":command": m["a"], ":type": TYPE_KW[3], ":resp-chan": chan}
    if typ == 4:
        return {":term": m["term"], ":id": src, ":type": TYPE_KW[4], ":vote-granted": bool(flag)}
    if flag:
        return {":term": m["term"], ":id": src, ":type": TYPE_KW[5], ":success": True,
                ":commit": m["a"], ":log-index": m["b"]}
    return {":term": m["term"], ":id": src, ":type": TYPE_KW[5], ":success": False}


def format_event(ev: dict, entries, node_id: int, n_nodes: int, set_order="sorted") -> str:
    return ("; Node\n" + edn(node_map(ev, node_id, n_nodes), set_order) + "\n; Message\n"
            + edn(message_map(ev, entries), set_order) + "\n\n")
