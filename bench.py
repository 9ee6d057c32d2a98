"""bench.py — simulated node-ticks/s of the batched Raft simulator on MI355X.

Headline workload (BASELINE.json configs[1], "C2"): 65,536 independent 5-node clusters per GPU, no
faults, no client traffic. One *step* = one raft_sim_step(10,000 ticks) over every cluster,
continuing the simulation; state is resident in HBM before timing starts. Under torchrun each rank
simulates its own 65,536 clusters (global ids rank*65536 + i: disjoint, shard-invariant Philox
streams; weak scaling, no data-path collective).

The same JSON line carries, under "workloads", BASELINE config 3 ("C3"): 1,048,576 five-node
clusters with 10 % drop, 1 % duplication, delay U[1,50], partitions and a bursty client that
follows redirects (SIM_SPEC D14/D15; one client-set per 100 ticks on average), timed the same way.
Under torchrun the 1M clusters are split across the ranks (strong scaling).

Per workload:
  roofline      the tick kernel against HBM bandwidth with the event model of DESIGN.md: per launch
                the hot node state in and out once (2 * S_node(N) bytes per node, S_node = 32 + 8N),
                64 B per delivered message (written and read once) and 16 B per appended log entry
                (read and written once), over the average launch time measured with HIP events on
                the simulator's stream. `traffic` is the PMC-measured HBM bytes per launch from
                pmc_traffic.json (scripts/summarize_profile.py), used only when it was measured on this kernel build
                (source hash match). SURVEY §8(d)'s per-node-tick formula, which charges the skipped
                idle ticks as if they moved state, is reported as `per_tick_model` (informational).
  cpu_baseline  the C oracle (oracle/raftref.c, the restatement of core.clj/log.clj; "port") on a
                bounded sample of the same workload, clusters mapped over host threads (the pmap
                analogue), with the same discrete-event idle-tick skipping the GPU kernel does;
                rank 0 at N=1 only. The every-tick restatement's rate is given beside it.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
TICKS_PER_STEP = 10000
FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
WORKLOADS = {
    # name: (config, clusters, per-rank scaling, CPU sample (clusters, steps), description)
    "c2": (dict(nodes=5, seed=42), 65536, "weak", (65536, 40),
           "C2: 65,536 five-node clusters per GPU x 10,000 ticks per step, no faults, no client"),
    "c3": (dict(nodes=5, seed=1, log_cap=256, client_ppm=80000, client_period=16384,
                client_burst=2048, client_redirects=4, **FAULTS), 1 << 20, "strong", (131072, 3),
           "C3: 1,048,576 five-node clusters across all GPUs x 10,000 ticks per step; drop 10 %, "
           "dup 1 %, delay U[1,50], partitions p=0.1 per 1000-tick epoch; client-sets in bursts "
           "(2048 of every 16384 ticks, 1 per 100 ticks on average) following up to 4 redirects"),
    "c4_n7": (dict(nodes=7, seed=3, log_cap=4096, client_ppm=500000, client_period=8192,
                   client_burst=2048, client_redirects=4), 16384, "weak", (16384, 2),
              "C4: 16,384 seven-node clusters, 4096-entry logs, bursty client (1000+-entry batches)"),
    "c4_n9": (dict(nodes=9, seed=5, log_cap=4096, client_ppm=500000, client_period=8192,
                   client_burst=2048, client_redirects=4), 16384, "weak", (16384, 2),
              "C4: 16,384 nine-node clusters, 4096-entry logs, bursty client (1000+-entry batches)"),
}
KERNEL_SOURCES = ["raft-simulation_amd/csrc/tick_kernel.hip", "raft-simulation_amd/csrc/device.hpp",
                  "raft-simulation_amd/csrc/raftsim.hip", "include/raftsim.h"]


def kernel_build_hash():
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()[:16]


def load_traffic(workload):
    """PMC HBM bytes per tick-kernel launch measured on THIS kernel source (else None)."""
    f = ROOT / "pmc_traffic.json"     # written by scripts/summarize_profile.py
    try:
        rec = json.loads(f.read_text()).get(workload)
    except (OSError, ValueError):
        return None
    if not rec or rec.get("kernel_src_sha") != kernel_build_hash():
        return None
    return rec.get("hbm_bytes_per_launch")


def cpu_baseline(cfg, sample, ticks=TICKS_PER_STEP):
    """The C oracle on `clusters` of the workload for `steps` steps after one warm-up step: with
    the GPU's discrete-event idle-tick skipping (value), and visiting every tick (informational,
    an eighth of the clusters for one step)."""
    import helpers

    clusters, steps = sample
    threads = helpers.cpu_threads()

    def rate(nc, k, skip):
        ref = helpers.oracle(n_clusters=nc, **cfg)
        helpers.oracle_threads(ref, threads)
        helpers.oracle_idle_skip(ref, skip)
        ref.step(ticks)                              # warm state, like the GPU's warm-up
        t0 = time.perf_counter()
        for _ in range(k):
            ref.step(ticks)
        dt = time.perf_counter() - t0
        return nc * cfg["nodes"] * ticks * k / dt, dt

    v, dt = rate(clusters, steps, True)
    v_every, dt_every = rate(max(1, clusters // 8), 1, False)
    return {"value": v, "unit": "node-ticks/s", "cores": threads, "kind": "port",
            "sample": f"{clusters} clusters x {cfg['nodes']} nodes x {steps} steps of {ticks} "
                      f"ticks after a warm-up step, oracle/raftref.c with the same idle-tick "
                      f"skipping as the kernel, {threads} threads, {dt:.2f} s",
            "every_tick_value": v_every,
            "every_tick_sample": f"{max(1, clusters // 8)} clusters x 1 step visiting every tick, "
                                 f"{dt_every:.2f} s"}


def run_workload(name, args, world, rank, local_rank, dist):
    import raftsim
    from raftsim import dist as rdist

    cfg, clusters, scaling, cpu_sample, desc = WORKLOADS[name]
    n = cfg["nodes"]
    if scaling == "weak":
        offset, count = rank * clusters, clusters
        total = clusters * world
    else:
        offset, count = rdist.shard(clusters, rank, world)
        total = clusters
    if args.clusters and name == args.workload.split("+")[0]:
        count, total = args.clusters, args.clusters * world
    sim = raftsim.Simulator(n_clusters=count, cluster_offset=offset, device=local_rank, **cfg)

    def sync():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        sim.step(TICKS_PER_STEP)
    c_before = sim.counters()
    sync()
    t0 = time.perf_counter()
    # K steps enqueued back to back on the simulator's stream (raft_sim_step_async), then one
    # raft_sim_sync: per-launch HIP events still time every tick-kernel launch of the K steps
    for _ in range(args.steps):
        sim.step_async(TICKS_PER_STEP)
    sim.sync()
    sync()
    elapsed = time.perf_counter() - t0
    avg_launch_ms, launches = sim.last_step_timing()
    c_after = sim.counters()
    delta = {k: c_after[k] - c_before[k] for k in c_after
             if k not in ("first_violation_tick", "payload_max")}
    delta["payload_max"] = c_after["payload_max"]
    delta["first_violation_tick"] = c_after["first_violation_tick"]
    import ctypes
    import numpy as np

    raw = sim.read_nodes_raw()
    rec_bytes = np.frombuffer(raw, dtype=np.uint8).reshape(len(raw), ctypes.sizeof(raw[0]))
    role, fault = rec_bytes[:, 0], rec_bytes[:, 3]      # raft_node_t.role, .fault
    leaders_now = int(((role == 2) & (fault == 0)).sum())
    halted_now = int((fault != 0).sum())
    elapsed_max = elapsed
    if dist is not None:
        dev = f"cuda:{local_rank}"
        elapsed_max = rdist.reduce_max(elapsed, dev)
        delta = rdist.reduce_counters(delta, dev)
        avg_launch_ms = rdist.reduce_max(avg_launch_ms, dev)
        leaders_now = int(rdist.reduce_max(float(leaders_now), dev))  # per-rank max, informational
    node_ticks = delta["node_ticks"]

    # event model (per launch of one rank's shard): hot state in + out, 64 B per delivered
    # message, 16 B per appended entry (counts are whole-job, divided back to one launch)
    total_launches = max(1, launches * world)
    s_node = 32 + 8 * n
    msgs = delta["delivered"] / total_launches
    entries = delta["entries_appended"] / total_launches
    event_bytes = 2 * s_node * count * n + 64 * msgs + 16 * entries
    achieved = event_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms else 0.0
    ticks_per_launch = args.steps * TICKS_PER_STEP / max(1, launches)
    nt = max(1, node_ticks)
    per_tick_b = 2 * s_node + 8 + 64 * delta["delivered"] / nt + 16 * delta["entries_appended"] / nt
    per_tick_gbs = per_tick_b * count * n * ticks_per_launch / (avg_launch_ms * 1e-3) / 1e9 \
        if avg_launch_ms else 0.0
    rec = {
        "value": node_ticks / elapsed_max,
        "unit": "node-ticks/s",
        "ms_per_step": elapsed_max * 1e3 / args.steps,
        "scaling": scaling,
        "config": {"workload": desc, "clusters": total, "clusters_per_gpu": count, "nodes": n,
                   "ticks_per_step": TICKS_PER_STEP,
                   "parallelism": f"cluster-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(name),
                     "model": "event: 2*S_node*nodes + 64 B/delivered msg + 16 B/appended entry "
                              "per launch",
                     "bytes_per_launch": event_bytes, "avg_launch_ms": avg_launch_ms,
                     "launches": launches, "ticks_per_launch": ticks_per_launch,
                     "kernel_src_sha": kernel_build_hash(),
                     "limiter": "issue of the active trips' divergent instruction stream "
                                "(PMC instruction counts, region counts: DESIGN.md), not HBM "
                                "bandwidth",
                     "per_tick_model": {"bytes_per_node_tick": per_tick_b,
                                        "achieved": per_tick_gbs,
                                        "note": "SURVEY 8(d) B(N) charged to every node-tick "
                                                "incl. the skipped idle ones"}},
        "counters": {k: v for k, v in delta.items() if v},
        "leaders_at_end": leaders_now, "halted_at_end": halted_now,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(cfg, cpu_sample)
    sim.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2+c3",
                    help="headline[+extra...] from " + ", ".join(WORKLOADS))
    ap.add_argument("--clusters", type=int, default=0, help="override the headline's clusters")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if "RANK" in os.environ and "MASTER_ADDR" in os.environ:     # launched by torchrun
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")                           # RCCL on ROCm

    names = args.workload.split("+")
    recs = {name: run_workload(name, args, world, rank, local_rank, dist) for name in names}
    if rank == 0:
        head = recs[names[0]]
        out = {
            "metric": "simulated node-ticks/sec (5-node Raft)" if WORKLOADS[names[0]][0]["nodes"] == 5
            else "simulated node-ticks/sec",
            "value": head["value"],
            "unit": "node-ticks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": head["scaling"],
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded Philox clusters from init-node state)",
            "config": head["config"],
            "roofline": head["roofline"],
            "counters": head["counters"],
        }
        if "cpu_baseline" in head:
            out["cpu_baseline"] = head["cpu_baseline"]
        if len(names) > 1:
            out["workloads"] = {name: recs[name] for name in names[1:]}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
