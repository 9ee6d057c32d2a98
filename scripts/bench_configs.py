"""BASELINE configs 3-5 on one MI355X next to the CPU oracle (one GPU call; a JSON line per result).

c3      one GPU's shard of config 3 (131,072 of the 1,048,576 five-node clusters): drop 10 %, dup 1 %,
        delay U[1,50], partitions (p 0.1 per 1000-tick epoch), bursty client (SIM_SPEC D14/D15) at
        one client-set per 100 ticks on average. bench.py times the whole 1M clusters.
c4_n7, c4_n9   config 4: 16,384 clusters of 7 / 9 nodes with 4096-entry logs and a bursty client
        (500,000 ppm in 2048 of every 8192 ticks, redirects followed) run for 110k ticks: log
        growth, 1000+-entry AppendEntries batches, OVERFLOW halts; kernel time per 10k-tick step.
c4_spec_n9     the same on the Spec-Raft control (majority commit through the sorting network).
c5      config 5: config 3's faults and client with the vote granted without the log check, on the
        faithful model (flag 1) and on the Spec-Raft control (flags 3); ticks until the first safety
        violation anywhere in the shard, GPU wall time next to the CPU oracle's on the same
        clusters (all host threads, idle-tick skipping), bit-exactness, and the Spec-Raft control
        (flag 2) run for as many ticks: leaders, commits, violations.
GPU rates are node-ticks/s over steps of 10k ticks after a warm-up (state resident in HBM)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import helpers  # noqa: E402
import raftsim  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
C3 = dict(nodes=5, seed=1, client_ppm=80000, client_period=16384, client_burst=2048,
          client_redirects=4, log_cap=256, **FAULTS)
C4 = dict(log_cap=4096, client_ppm=500000, client_period=8192, client_burst=2048,
          client_redirects=4)


def emit(rec):
    print(json.dumps(rec), flush=True)


def cpu_oracle(cfg, clusters, ticks_list):
    r = helpers.oracle(n_clusters=clusters, **cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    helpers.oracle_idle_skip(r)
    dts = []
    for t in ticks_list:
        t0 = time.perf_counter()
        r.step(t)
        dts.append(time.perf_counter() - t0)
    return r, dts


def node_census(sim):
    import ctypes
    raw = sim.read_nodes_raw()
    b = np.frombuffer(raw, dtype=np.uint8).reshape(len(raw), ctypes.sizeof(raw[0]))
    log_len = b[:, 20:24].copy().view(np.uint32).ravel()
    return {"leaders_running": int(((b[:, 0] == 2) & (b[:, 3] == 0)).sum()),
            "halted_nodes": int((b[:, 3] != 0).sum()), "max_log_len": int(log_len.max())}


def c3_shard():
    n, clusters = 5, 131072
    g = raftsim.Simulator(n_clusters=clusters, **C3)
    g.step(20000)
    t0 = time.perf_counter()
    for _ in range(4):
        g.step(10000)
    gdt = time.perf_counter() - t0
    _, dts = cpu_oracle(C3, 8192, [20000, 40000])
    emit({"config": "c3_shard", "gpu_clusters": clusters,
          "gpu_node_ticks_per_s": clusters * n * 40000 / gdt,
          "cpu_clusters": 8192, "cpu_threads": helpers.cpu_threads(),
          "cpu_node_ticks_per_s": 8192 * n * 40000 / dts[1],
          "gpu_counters": {k: v for k, v in g.counters().items() if v}, **node_census(g)})


def c4(name, nodes, seed, variant=0, clusters=16384, total=110000):
    cfg = dict(nodes=nodes, seed=seed, variant_flags=variant, **C4)
    g = raftsim.Simulator(n_clusters=clusters, **cfg)
    steps, kms = [], []
    t_all = time.perf_counter()
    for s in range(total // 10000):
        t0 = time.perf_counter()
        g.step(10000)
        steps.append(time.perf_counter() - t0)
        kms.append(g.last_step_timing()[0])
    gdt = time.perf_counter() - t_all
    cpu_n = 512
    r, dts = cpu_oracle(cfg, cpu_n, [total])
    same = bool((g.digest(0, cpu_n) == r.digest()).all())
    emit({"config": name, "variant_flags": variant, "clusters": clusters, "ticks": total,
          "gpu_node_ticks_per_s": clusters * nodes * total / gdt,
          "kernel_ms_per_10k_ticks": [round(x, 3) for x in kms],
          "cpu_clusters": cpu_n, "cpu_threads": helpers.cpu_threads(),
          "cpu_node_ticks_per_s": cpu_n * nodes * total / dts[0], "first_clusters_bit_exact": same,
          "gpu_counters": {k: v for k, v in g.counters().items() if v}, **node_census(g)})


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


def time_to_violation(name, flags, clusters=131072, chunk=1000, max_ticks=200000):
    cfg = dict(C3, variant_flags=flags)
    g = raftsim.Simulator(n_clusters=clusters, **cfg)
    gfv, gdone, gdt = first_violation(g, chunk, max_ticks)
    r = helpers.oracle(n_clusters=clusters, **cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    helpers.oracle_idle_skip(r)
    cfv, cdone, cdt = first_violation(r, chunk, gdone)
    emit({"config": name, "variant_flags": flags, "clusters": clusters,
          "first_violation_tick": gfv, "ticks_simulated": gdone, "gpu_wall_s": gdt,
          "cpu_first_violation_tick": cfv, "cpu_wall_s": cdt, "cpu_threads": helpers.cpu_threads(),
          "bit_exact": bool(gfv == cfv and cdone == gdone and (g.digest() == r.digest()).all()),
          "gpu_counters": {k: v for k, v in g.counters().items() if v}})
    return gdone


def main():
    names = sys.argv[1:] or ["c3", "c4", "c5"]
    if "c3" in names:
        c3_shard()
    if "c4" in names:
        c4("c4_n7", 7, 3)
        c4("c4_n9", 9, 5)
        c4("c4_spec_n9", 9, 5, variant=2)
    if "c5" in names:
        ticks = time_to_violation("c5_faithful_nolog", 1)
        ticks = max(ticks, time_to_violation("c5_spec_nolog", 3))
        ctl = raftsim.Simulator(n_clusters=131072, **dict(C3, variant_flags=2))
        t0 = time.perf_counter()
        ctl.step(ticks)
        c = ctl.counters()
        emit({"config": "c5_spec_control", "variant_flags": 2, "clusters": 131072,
              "ticks_simulated": ticks, "gpu_wall_s": time.perf_counter() - t0,
              "first_violation_tick": c["first_violation_tick"], "leaders": c["leaders"],
              "entries_applied": c["entries_applied"],
              "violations": c["viol_election"] + c["viol_log"] + c["viol_complete"],
              **node_census(ctl)})


if __name__ == "__main__":
    main()
