"""Regenerate the golden fixtures from the Python restatement (oracle/pyref.py).

The reference itself cannot run here (Clojure 1.6 on a JVM; no JVM in this image), so the fixtures
are the Python restatement's outputs: per-event traces and final canonical states for small seeded
runs. tests/test_golden.py checks the C oracle (CPU) and libraftsim.so (GPU) against them.
Run: python tests/golden/make_golden.py
"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import pyref  # noqa: E402

CASES = {
    # BASELINE config 1: single 5-node cluster, seed 42, 10k ticks, no faults (full event trace)
    "c1_seed42": dict(cfg=dict(nodes=5, seed=42), gid=0, ticks=10000, trace=True, stdout=True),
    "c1_seed1": dict(cfg=dict(nodes=5, seed=1), gid=0, ticks=10000, trace=True, stdout=True),
    "faults_n5": dict(cfg=dict(nodes=5, seed=7, drop_ppm=100000, dup_ppm=20000, dmin=1, dmax=30,
                               part_ppm=100000, client_ppm=1500, log_cap=128), gid=3,
                      ticks=30000, trace=True),
    "client_n7": dict(cfg=dict(nodes=7, seed=11, client_ppm=3000, log_cap=256), gid=5,
                      ticks=20000, trace=False),
    "overflow_n9": dict(cfg=dict(nodes=9, seed=13, inbox_cap=2, dup_ppm=300000, dmax=3,
                                 client_ppm=5000, log_cap=64), gid=1, ticks=20000, trace=False),
    "variant_n3": dict(cfg=dict(nodes=3, seed=17, variant_flags=1, client_ppm=150,
                                drop_ppm=50000, log_cap=64), gid=2, ticks=30000, trace=False),
    # BASELINE config 4 shape: 7 nodes, 4096-entry logs, bursty client traffic that follows
    # redirect-client to the leader (SIM_SPEC D14/D15): multi-thousand-entry AppendEntries batches
    "c4_bursts_n7": dict(cfg=dict(nodes=7, seed=3, log_cap=4096, client_ppm=500000,
                                  client_period=8192, client_burst=2048, client_redirects=4),
                         gid=5, ticks=36000, trace=False),
    # config 3 faults with bursts and redirects on 5 nodes, full event trace
    "c3_bursts_n5": dict(cfg=dict(nodes=5, seed=1, drop_ppm=100000, dup_ppm=10000, dmin=1,
                                  dmax=50, part_ppm=100000, log_cap=256, client_ppm=80000,
                                  client_period=16384, client_burst=2048, client_redirects=4),
                         gid=9, ticks=40000, trace=True),
    # F4 Spec-Raft control (SIM_SPEC §8) with faults and client traffic, full event trace
    "spec_n5": dict(cfg=dict(nodes=5, seed=19, variant_flags=2, client_ppm=2000, drop_ppm=100000,
                             dup_ppm=20000, dmin=1, dmax=30, part_ppm=100000, log_cap=256,
                             hb=300, el_base=500, el_span=500), gid=4, ticks=30000, trace=True),
    "spec_bursts_n5": dict(cfg=dict(nodes=5, seed=23, variant_flags=2, drop_ppm=100000,
                                    dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000, log_cap=1024,
                                    client_ppm=200000, client_period=8192, client_burst=1024,
                                    client_redirects=4), gid=6, ticks=40000, trace=True),
}


class Tracer(pyref.PyCluster):
    """PyCluster that records (tick, node, trace-hash) whenever a node's trace hash changes."""

    def step(self, t):
        before = dict(self.trace)
        super().step(t)
        for i in sorted(self.trace):
            if self.trace[i] != before[i]:
                n = self.canonical_node(i)
                self.hash_events.append([t, i, n["role"], n["current_term"], n["fault"],
                                         format(self.trace[i], "016x")])


def make(name, spec):
    cfg = pyref.default_config(**spec["cfg"], trace_cap=1 if spec.get("stdout") else 0)
    c = Tracer(cfg, spec["gid"])
    c.hash_events = []
    for t in range(spec["ticks"]):
        c.step(t)
    nodes = []
    for i in range(1, c.N + 1):
        n = c.canonical_node(i)
        n["trace_hash"] = format(n["trace_hash"], "016x")
        n["log"] = [list(e) for e in c.logs[i].entries]
        n["req"] = [list(m[:7]) + [[list(e) for e in m[7]]] for m in c.canonical_msgs(i, 0)]
        n["res"] = [list(m[:7]) + [[list(e) for e in m[7]]] for m in c.canonical_msgs(i, 1)]
        nodes.append(n)
    out = {"config": spec["cfg"], "cluster_offset": spec["gid"], "ticks": spec["ticks"],
           "nodes": nodes, "hwm": list(c.hwm), "client": [c.client_next, c.client_count],
           "counters": c.cnt, "payload_max": c.payload_max,
           "first_violation_tick": c.first_violation}
    if spec["trace"]:
        out["events"] = c.hash_events
    if spec.get("stdout"):      # F3: what each node's `wait` prints (core.clj:182-186)
        out["stdout"] = {str(i): pyref.stdout_of(c, i) for i in range(1, c.N + 1)}
    (HERE / f"{name}.json").write_text(json.dumps(out, separators=(",", ":")) + "\n")
    return out


if __name__ == "__main__":
    for name, spec in CASES.items():
        o = make(name, spec)
        print(name, {k: v for k, v in o["counters"].items() if v})
