"""bench.py — simulated node-ticks/s of the batched 5-node Raft simulator on MI355X.

Workload (BASELINE.json configs[1], "C2"): 65,536 independent 5-node clusters per GPU, no faults,
no client traffic. One *step* = one raft_sim_step(10,000 ticks) over every cluster (the config's
10k-tick run), continuing the simulation. Inputs/state are resident in HBM before timing starts.
Multi-GPU (torchrun): each rank simulates its own 65,536 clusters (global ids rank*65536 + i, so
Philox streams are disjoint and shard-invariant: weak scaling, no data-path collective); the
counters and the per-rank times are all-reduced over RCCL (torch.distributed, backend "nccl").

The JSON line also carries:
  roofline      the tick kernel against HBM bandwidth using SURVEY.md §8(d)'s algorithmic bytes
                B(N) = 2·(32+8N) + 8 + 64·m + 16·e per node-tick (m = messages delivered and
                e = log entries appended per node-tick, from this run's counters), divided by the
                average launch duration measured with HIP events on the simulator's stream.
                `traffic` is the PMC-measured HBM bytes per launch from profiles/ when present.
  cpu_baseline  the C oracle (oracle/raftref.c, the restatement of core.clj/log.clj; "port") on a
                bounded sample of the same workload, clusters mapped over host threads (the pmap
                analogue), rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
CLUSTERS_PER_GPU = 65536
NODES = 5
TICKS_PER_STEP = 10000


def algorithmic_bytes_per_node_tick(n, counters):
    nt = max(1, counters["node_ticks"])
    m = counters["delivered"] / nt
    e = counters["entries_appended"] / nt
    return 2 * (32 + 8 * n) + 8 + 64 * m + 16 * e, m, e


def cpu_baseline(seed):
    import helpers

    threads = helpers.cpu_threads()
    clusters = min(CLUSTERS_PER_GPU, 4096 * threads)
    ticks = TICKS_PER_STEP
    ref = helpers.oracle(n_clusters=clusters, nodes=NODES, seed=seed)
    helpers.oracle_threads(ref, threads)
    t0 = time.perf_counter()
    ref.step(ticks)
    dt = time.perf_counter() - t0
    return {"value": clusters * NODES * ticks / dt, "unit": "node-ticks/s", "cores": threads,
            "kind": "port",
            "sample": f"{clusters} clusters x {NODES} nodes x {ticks} ticks (C2 shape), "
                      f"oracle/raftref.c, {threads} threads, {dt:.2f} s"}


def load_traffic():
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clusters", type=int, default=CLUSTERS_PER_GPU)
    ap.add_argument("--ticks-per-launch", type=int, default=0)
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

    import raftsim

    sim = raftsim.Simulator(n_clusters=args.clusters, cluster_offset=rank * args.clusters,
                            nodes=NODES, seed=42, device=local_rank if world > 1 else 0,
                            ticks_per_launch=args.ticks_per_launch)

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
    # raft_sim_sync: the host does not wait between steps; per-launch HIP events still time
    # every tick-kernel launch of the K steps
    for _ in range(args.steps):
        sim.step_async(TICKS_PER_STEP)
    sim.sync()
    ms, launches = sim.last_step_timing()
    kernel_ms = ms * launches
    sync()
    elapsed = time.perf_counter() - t0
    c_after = sim.counters()
    delta = {k: (c_after[k] - c_before[k]) for k in c_after if k != "first_violation_tick"}

    elapsed_max = elapsed
    if dist is not None:
        from raftsim import dist as rdist

        dev = f"cuda:{local_rank}"
        elapsed_max = rdist.reduce_max(elapsed, dev)
        delta = rdist.reduce_counters(dict(delta, first_violation_tick=None), dev)
        kernel_ms = rdist.reduce_max(kernel_ms, dev)
    total_node_ticks = delta["node_ticks"]

    if rank == 0:
        bpnt, m, e = algorithmic_bytes_per_node_tick(NODES, delta)
        avg_launch_ms = kernel_ms / max(1, launches)
        ticks_per_launch = args.steps * TICKS_PER_STEP / max(1, launches)
        node_ticks_per_launch = args.clusters * NODES * ticks_per_launch
        achieved = bpnt * node_ticks_per_launch / (avg_launch_ms * 1e-3) / 1e9
        # The fused kernel's own minimum HBM traffic per launch: hot node state in and out once
        # (S_node(N) = 32 + 8N bytes each way), plus every message written to and read from a
        # queue (64 B) and every log entry copied (16 B) -- what a perfect implementation of THIS
        # design must move; compare with `traffic` (PMC) and with the peak.
        launch_share = node_ticks_per_launch / max(1, total_node_ticks)
        fused_bytes = (2 * (32 + 8 * NODES) * args.clusters
                       + (64 * delta["delivered"] + 16 * delta["entries_appended"]) * launch_share)
        fused_gbs = fused_bytes / (avg_launch_ms * 1e-3) / 1e9
        value = total_node_ticks / elapsed_max
        out = {
            "metric": "simulated node-ticks/sec (5-node Raft)",
            "value": value,
            "unit": "node-ticks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded Philox clusters from init-node state)",
            "config": {"workload": "C2: 65,536 five-node clusters per GPU x 10,000 ticks per "
                                   "step, no faults, no client-set",
                       "clusters_per_gpu": args.clusters, "nodes": NODES,
                       "ticks_per_step": TICKS_PER_STEP,
                       "parallelism": f"cluster-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": load_traffic(),
                         "algorithmic_bytes_per_node_tick": bpnt,
                         "msgs_per_node_tick": m, "entries_per_node_tick": e,
                         "avg_launch_ms": avg_launch_ms, "ticks_per_launch": ticks_per_launch,
                         "fused_model": {"bytes_per_launch": fused_bytes, "achieved": fused_gbs,
                                         "frac": fused_gbs / HBM_PEAK_GBS}},
            "counters": {k: v for k, v in delta.items() if v and k != "first_violation_tick"},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(42)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
