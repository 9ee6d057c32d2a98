"""Compare a backend against a golden fixture of tests/golden/ (test infrastructure)."""
import json
from pathlib import Path

GOLDEN = Path(__file__).resolve().parent / "golden"
NAMES = sorted(p.stem for p in GOLDEN.glob("*.json"))
FIELDS = ["role", "voted_for", "leader_id", "fault", "entries_is_seq", "ls_present", "votes",
          "ls_keys", "current_term", "commit_index", "log_len", "deadline", "next_index",
          "match_index", "last_led_term", "req_count", "res_count", "commit_count"]


def load(name):
    return json.loads((GOLDEN / f"{name}.json").read_text())


def check(name, make):
    fx = load(name)
    cfg = dict(fx["config"], n_clusters=1, cluster_offset=fx["cluster_offset"])
    if "stdout" in fx:
        cfg.update(trace_cap=4096, trace_entry_cap=1 << 16)
    be = make(**cfg)
    N = cfg["nodes"]
    if "events" in fx:
        events, prev = [], [r["trace_hash"] for r in be.read_nodes(0, 1)]
        for t in range(fx["ticks"]):
            be.step(1)
            recs = be.read_nodes(0, 1)
            for i, r in enumerate(recs):
                if r["trace_hash"] != prev[i]:
                    events.append([t, i + 1, r["role"], r["current_term"], r["fault"],
                                   format(r["trace_hash"], "016x")])
            prev = [r["trace_hash"] for r in recs]
        assert events == fx["events"], _first_diff(events, fx["events"])
    else:
        be.step(fx["ticks"])
    recs = be.read_nodes(0, 1)
    for i in range(N):
        want, got = fx["nodes"][i], recs[i]
        for f in FIELDS:
            assert got[f] == want[f], (name, i + 1, f, got[f], want[f])
        assert format(got["trace_hash"], "016x") == want["trace_hash"], (name, i + 1)
        assert [list(e) for e in be.log(0, i + 1)] == want["log"], (name, i + 1, "log")
        for which, key in ((0, "req"), (1, "res")):
            q = be.read_queue(0, i + 1, which)
            assert [list(m[:7]) for m in q] == [m[:7] for m in want[key]], (name, i + 1, key)
            for m, w in zip(q, want[key]):
                pcnt = m[1] >> 16
                if pcnt:
                    ar = be.read_arena(0, (m[1] >> 3) & 15)
                    got_p = [list(ar[(m[7] + k) % len(ar)]) for k in range(pcnt)]
                    assert got_p == w[7], (name, i + 1, "payload")
    cr = be.read_clusters(0, 1)[0]
    assert list(cr["hwm"]) == fx["hwm"]
    assert [cr["client_next"], cr["client_count"]] == fx["client"]
    c = be.counters()
    for k, v in fx["counters"].items():
        assert c[k] == v, (name, k, c[k], v)
    assert c["first_violation_tick"] == fx["first_violation_tick"]
    if "payload_max" in fx:
        assert c["payload_max"] == fx["payload_max"], (name, c["payload_max"], fx["payload_max"])
    for i, text in fx.get("stdout", {}).items():
        assert be.edn_trace(0, int(i)) == text, (name, "stdout of node", i)


def _first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return f"event {i}: got {x} want {y}"
    return f"lengths {len(a)} vs {len(b)}"
