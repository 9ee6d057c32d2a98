"""BASELINE configs 3-5 on one MI355X next to the CPU oracle (one GPU call; JSON line per result).

c3     one GPU's shard of config 3 (131,072 of the 1,048,576 five-node clusters): 10 % drop, dup 1 %,
       delay U[1,50], partitions (p 0.1 per 1000-tick epoch), one client-set per 100 ticks.
c4_n7, c4_n9   16,384 clusters with 4096-entry logs and a client-set every 4 ticks.
c5_*   config 5: config 3's faults with the vote granted without the log check (flag 1), on the
       faithful model and on the Spec-Raft control (flags 3); ticks until the first safety violation
       anywhere in the shard, GPU wall time next to the CPU oracle's on the same clusters, and the
       Spec-Raft control (flag 2) run for as many ticks with no violation.
GPU rates are node-ticks/s over a 10k-tick step after a 10k-tick warm-up (state resident in HBM);
the CPU oracle runs a fixed subset with all host threads (the pmap analogue)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import helpers  # noqa: E402
import raftsim  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
C3 = dict(nodes=5, seed=1, client_ppm=10000, log_cap=256, **FAULTS)
THROUGHPUT = {
    "c3": (C3, 131072, 4096),
    "c4_n7": (dict(nodes=7, seed=3, client_ppm=250000, log_cap=4096), 16384, 256),
    "c4_n9": (dict(nodes=9, seed=5, client_ppm=250000, log_cap=4096), 16384, 256),
}


def emit(rec):
    print(json.dumps(rec), flush=True)


def throughput(name, cfg, clusters, cpu_clusters, ticks=10000):
    g = raftsim.Simulator(n_clusters=clusters, **cfg)
    g.step(ticks)
    t0 = time.perf_counter()
    g.step(ticks)
    gdt = time.perf_counter() - t0
    ms, _ = g.last_step_timing()
    r = helpers.oracle(n_clusters=cpu_clusters, **cfg)
    threads = helpers.cpu_threads()
    helpers.oracle_threads(r, threads)
    r.step(ticks)
    t0 = time.perf_counter()
    r.step(ticks)
    cdt = time.perf_counter() - t0
    n = cfg["nodes"]
    emit({"config": name, "gpu_clusters": clusters, "gpu_node_ticks_per_s": clusters * n * ticks / gdt,
          "kernel_ms_per_10k_ticks": ms, "cpu_clusters": cpu_clusters, "cpu_threads": threads,
          "cpu_node_ticks_per_s": cpu_clusters * n * ticks / cdt,
          "gpu_counters": {k: v for k, v in g.counters().items() if v}})


def first_violation(sim, chunk, max_ticks):
    t0 = time.perf_counter()
    done = 0
    while done < max_ticks:
        sim.step(chunk)
        done += chunk
        fv = sim.counters()["first_violation_tick"]
        if fv is not None:
            return fv, done, time.perf_counter() - t0
    return None, done, time.perf_counter() - t0


def time_to_violation(name, flags, clusters=131072, chunk=500, max_ticks=100000):
    cfg = dict(C3, variant_flags=flags)
    g = raftsim.Simulator(n_clusters=clusters, **cfg)
    gfv, gdone, gdt = first_violation(g, chunk, max_ticks)
    r = helpers.oracle(n_clusters=clusters, **cfg)
    threads = helpers.cpu_threads()
    helpers.oracle_threads(r, threads)
    cfv, cdone, cdt = first_violation(r, chunk, gdone)
    emit({"config": name, "variant_flags": flags, "clusters": clusters,
          "first_violation_tick": gfv, "ticks_simulated": gdone, "gpu_wall_s": gdt,
          "cpu_first_violation_tick": cfv, "cpu_wall_s": cdt, "cpu_threads": threads,
          "bit_exact": bool(gfv == cfv and cdone == gdone and (g.digest() == r.digest()).all())})
    return gdone


def main():
    names = sys.argv[1:] or ["c3", "c4_n7", "c4_n9", "c5"]
    for name in names:
        if name in THROUGHPUT:
            cfg, clusters, cpu_clusters = THROUGHPUT[name]
            throughput(name, cfg, clusters, cpu_clusters)
        elif name == "c5":
            ticks = time_to_violation("c5_faithful_nolog", 1)
            ticks = max(ticks, time_to_violation("c5_spec_nolog", 3))
            ctl = raftsim.Simulator(n_clusters=131072, **dict(C3, variant_flags=2))
            ctl.step(ticks)
            c = ctl.counters()
            emit({"config": "c5_spec_control", "variant_flags": 2, "clusters": 131072,
                  "ticks_simulated": ticks, "first_violation_tick": c["first_violation_tick"],
                  "leaders": c["leaders"], "entries_applied": c["entries_applied"],
                  "violations": c["viol_election"] + c["viol_log"] + c["viol_complete"]})


if __name__ == "__main__":
    main()
