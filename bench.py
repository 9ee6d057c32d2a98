"""bench.py — simulated node-ticks/s of the batched Raft simulator on MI355X.

Headline workload (BASELINE.json configs[1], "C2"): 65,536 independent 5-node clusters per GPU, no
faults, no client traffic. One *step* = one raft_sim_step(10,000 ticks) over every cluster,
continuing the simulation; state is resident in HBM before timing starts. Under torchrun each rank
simulates its own 65,536 clusters (global ids rank*65536 + i: disjoint, shard-invariant Philox
streams; weak scaling, no data-path collective). C2 is periodic in steady state (heartbeat rounds
every hb ticks), so its window is the K steps after W warm-up steps.

The same JSON line carries, under "workloads", BASELINE config 3 ("C3"): 1,048,576 five-node
clusters with 10 % drop, 1 % duplication, delay U[1,50], partitions and a bursty client that
follows redirects (SIM_SPEC D14/D15; one client-set per 100 ticks on average), and the same traffic
under the Spec-Raft control ("C3-spec", SIM_SPEC §8: no crash storm, real replication at 1M
clusters). Under the faithful handlers C3 turns into a crash storm whose cost per tick changes as
nodes halt, so the C3 windows are fixed: ticks [0, 10,000 K) from init-node on a fresh handle (the
W warm-up steps run on a throwaway handle of the same shape), and the line reports the live-node
fraction at the window's end and the live node-ticks/s. Under torchrun the 1M clusters are split
across the ranks (strong scaling).

Per workload:
  roofline      the tick kernel against HBM bandwidth with the event model of DESIGN.md: per launch
                the hot node state in and out once (2 * S_node(N) bytes per node, S_node = 32 + 8N),
                64 B per delivered message (written and read once) and 16 B per appended log entry
                (read and written once), over the average launch time measured with HIP events on
                the simulator's stream. `traffic` is the PMC-measured HBM bytes per launch from
                pmc_traffic.json (scripts/summarize_profile.py), used only when it was measured on
                this kernel build (source hash) over this same window (steps, warm-up, window kind).
                `bound` is the roofline axis (HBM); the measured limiter is named in `limiter`.
                `frac_state_model` prices only the hot state in and out: a C2 launch on the
                lane-per-cluster steady kernel keeps its messages in registers, so the event
                model's 64 B per message is not HBM traffic there (PMC `traffic` shows it).
  cpu_baseline  the C oracle (oracle/raftref.c, the restatement of core.clj/log.clj; "port") on a
                bounded sample of the same workload over the same tick window, clusters mapped over
                every host CPU this process may run on (the pmap analogue), with the same
                discrete-event idle-tick skipping the GPU kernel does; rank 0 at N=1 only. The
                every-tick restatement's rate is given beside it.
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
C3_CFG = dict(nodes=5, seed=1, log_cap=256, client_ppm=80000, client_period=16384,
              client_burst=2048, client_redirects=4, **FAULTS)
C3_DESC = ("1,048,576 five-node clusters across all GPUs x 10,000 ticks per step; drop 10 %, dup 1 "
           "%, delay U[1,50], partitions p=0.1 per 1000-tick epoch; client-sets in bursts (2048 of "
           "every 16384 ticks, 1 per 100 ticks on average) following up to 4 redirects; window: "
           "ticks [0, 10000 * steps) from init-node")
# name: config, clusters, per-rank scaling, window, CPU sample, description. CPU sample: (clusters,
# steps) after a warm-up step for "steady" windows; for "init" windows cluster-steps, i.e. the
# oracle runs cluster_steps // steps clusters over the GPU's own window from init-node.
WORKLOADS = {
    "c2": dict(cfg=dict(nodes=5, seed=42), clusters=65536, scaling="weak", window="steady",
               cpu=(65536, 40),
               desc="C2: 65,536 five-node clusters per GPU x 10,000 ticks per step, no faults, "
                    "no client"),
    "c3": dict(cfg=C3_CFG, clusters=1 << 20, scaling="strong", window="init", cpu=1 << 19,
               desc="C3: " + C3_DESC),
    "c3_spec": dict(cfg=dict(C3_CFG, variant_flags=2, log_cap=1024), clusters=1 << 20,
                    scaling="strong", window="init", cpu=1 << 19,
                    desc="C3 under the Spec-Raft control (SIM_SPEC §8, 1024-entry logs): "
                         + C3_DESC),
    "c4_n7": dict(cfg=dict(nodes=7, seed=3, log_cap=4096, client_ppm=500000, client_period=8192,
                           client_burst=2048, client_redirects=4),
                  clusters=16384, scaling="weak", window="steady", cpu=(16384, 2),
                  desc="C4: 16,384 seven-node clusters, 4096-entry logs, bursty client "
                       "(1000+-entry batches)"),
    "c4_n9": dict(cfg=dict(nodes=9, seed=5, log_cap=4096, client_ppm=500000, client_period=8192,
                           client_burst=2048, client_redirects=4),
                  clusters=16384, scaling="weak", window="steady", cpu=(16384, 2),
                  desc="C4: 16,384 nine-node clusters, 4096-entry logs, bursty client "
                       "(1000+-entry batches)"),
}
KERNEL_SOURCES = ["raft-simulation_amd/csrc/tick_kernel.hip", "raft-simulation_amd/csrc/steady_kernel.hip",
                  "raft-simulation_amd/csrc/device.hpp",
                  "raft-simulation_amd/csrc/raftsim.hip", "include/raftsim.h"]
HALTS = ("halt_ioobe", "halt_npe", "halt_cce", "halt_overflow")
LIMITER = {
    "c2": "one wave per SIMD running 64 clusters' heartbeat rounds: the chain of dependent "
          "quarter-rate multiplies (Philox draws, FNV trace hash) per trip, then the state load "
          "and the write-back's per-lane L2 requests (per-wave timeline, DESIGN.md); messages stay "
          "in registers, so the event model's message bytes are not HBM traffic (see "
          "frac_state_model and traffic)",
    "c3": "issue of the active trips' divergent instruction stream (client-set injections and "
          "redirect hops, most of them into halted nodes; PMC instruction counts, DESIGN.md), not "
          "HBM bandwidth",
}


def kernel_build_hash():
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()[:16]


def window_id(spec, args):
    """The tick window a number describes: steady windows are the K steps after W warm-up steps
    (periodic state: any K), init windows ticks [0, 10000 K) from init-node."""
    if spec["window"] == "init":
        return {"kind": "init", "steps": args.steps}
    return {"kind": "steady", "steps": args.steps, "warmup": args.warmup}


def load_traffic(workload, window):
    """PMC HBM bytes per tick-kernel launch measured on THIS kernel source over this window (else
    None, with the reason)."""
    f = ROOT / "pmc_traffic.json"     # written by scripts/summarize_profile.py
    try:
        rec = json.loads(f.read_text()).get(workload)
    except (OSError, ValueError):
        return None, "no pmc_traffic.json"
    if not rec:
        return None, f"no PMC profile of {workload}"
    if rec.get("kernel_src_sha") != kernel_build_hash():
        return None, "PMC profile of another kernel build"
    if window["kind"] == "init" and rec.get("window") != window:
        return None, f"PMC profile window {rec.get('window')} is not this window"
    return rec.get("hbm_bytes_per_launch"), rec.get("source")


def host_cpus():
    """CPUs this process may run on (affinity), the machine's count, and the cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "nproc": os.cpu_count(), "cgroup_quota_cpus": quota}


def cpu_baseline(spec, args):
    """The C oracle over the GPU run's own tick window, on a bounded sample of its clusters, with
    the GPU's discrete-event idle-tick skipping (value); the every-tick restatement on an eighth
    of the sample for one step (informational)."""
    import helpers

    cfg = spec["cfg"]
    hc = host_cpus()
    threads = helpers.cpu_threads()     # the affinity mask capped by the cgroup CPU quota
    if spec["window"] == "init":
        steps = args.steps
        clusters = max(1024, min(spec["clusters"], spec["cpu"] // max(1, steps)))
    else:
        clusters, steps = spec["cpu"]

    def rate(nc, k, skip, warm):
        ref = helpers.oracle(n_clusters=nc, **cfg)
        helpers.oracle_threads(ref, threads)
        helpers.oracle_idle_skip(ref, skip)
        if warm:
            ref.step(TICKS_PER_STEP)               # warm state, like the GPU's warm-up
        t0 = time.perf_counter()
        for _ in range(k):
            ref.step(TICKS_PER_STEP)
        dt = time.perf_counter() - t0
        return nc * cfg["nodes"] * TICKS_PER_STEP * k / dt, dt

    warm = spec["window"] == "steady"
    v, dt = rate(clusters, steps, True, warm)
    v_every, dt_every = rate(max(1, clusters // 8), 1, False, warm)
    where = (f"ticks [0, {steps * TICKS_PER_STEP}) from init-node (the GPU's window)"
             if not warm else f"{steps} steps after a warm-up step")
    return {"value": v, "unit": "node-ticks/s", "cores": threads, "kind": "port",
            "sample": f"{clusters} clusters x {cfg['nodes']} nodes, {where}, oracle/raftref.c "
                      f"with the same idle-tick skipping as the kernel, {threads} threads (the host "
                      f"CPUs this process may use: affinity mask capped by the cgroup quota), "
                      f"{dt:.2f} s",
            "host_cpus": hc,
            "every_tick_value": v_every,
            "every_tick_sample": f"{max(1, clusters // 8)} clusters x 1 step visiting every tick, "
                                 f"{dt_every:.2f} s"}


def run_workload(name, args, world, rank, local_rank, dist):
    import raftsim
    from raftsim import dist as rdist

    spec = WORKLOADS[name]
    cfg, clusters, scaling = spec["cfg"], spec["clusters"], spec["scaling"]
    n = cfg["nodes"]
    if args.clusters and name == args.workload.split("+")[0]:
        clusters = args.clusters
    if scaling == "weak":
        offset, count = rank * clusters, clusters
        total = clusters * world
    else:
        offset, count = rdist.shard(clusters, rank, world)
        total = clusters

    def make():
        return raftsim.Simulator(n_clusters=count, cluster_offset=offset, device=local_rank, **cfg)

    def sync():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    init = spec["window"] == "init"
    if init:
        if args.warmup:                    # same shape, thrown away: the window starts at init
            w = make()
            for _ in range(args.warmup):
                w.step(TICKS_PER_STEP)
            w.sync()
            w.close()
        sim = make()
    else:
        sim = make()
        for _ in range(args.warmup):
            sim.step(TICKS_PER_STEP)
    c_before = sim.counters()
    nodes = count * n
    live = [nodes - sum(c_before[h] for h in HALTS)]
    sync()
    t0 = time.perf_counter()
    kernel_ms, launches = 0.0, 0
    if init:
        # one sync per step: the live-node count after every step (halts are permanent, so the
        # halt counters count the halted nodes) for the live node-ticks of the window
        for _ in range(args.steps):
            sim.step_async(TICKS_PER_STEP)
            sim.sync()
            ms, nl = sim.last_step_timing()
            kernel_ms += ms * nl
            launches += nl
            c = sim.counters()
            live.append(nodes - sum(c[h] for h in HALTS))
    else:
        # K steps enqueued back to back on the simulator's stream (raft_sim_step_async), then one
        # raft_sim_sync: per-launch HIP events still time every tick-kernel launch of the K steps
        for _ in range(args.steps):
            sim.step_async(TICKS_PER_STEP)
        sim.sync()
        ms, launches = sim.last_step_timing()
        kernel_ms = ms * launches
    sync()
    elapsed = time.perf_counter() - t0
    avg_launch_ms = kernel_ms / max(1, launches)
    c_after = sim.counters()
    if not init:
        live.append(nodes - sum(c_after[h] for h in HALTS))
    delta = {k: c_after[k] - c_before[k] for k in c_after
             if k not in ("first_violation_tick", "payload_max")}
    delta["payload_max"] = c_after["payload_max"]
    delta["first_violation_tick"] = c_after["first_violation_tick"]
    live_ticks = sum((a + b) / 2 for a, b in zip(live, live[1:])) * TICKS_PER_STEP \
        if init else (live[0] + live[-1]) / 2 * TICKS_PER_STEP * args.steps
    elapsed_max = elapsed
    if dist is not None:
        dev = f"cuda:{local_rank}"
        elapsed_max = rdist.reduce_max(elapsed, dev)
        delta = rdist.reduce_counters(delta, dev)
        avg_launch_ms = rdist.reduce_max(avg_launch_ms, dev)
        live_ticks = rdist.reduce_sum(live_ticks, dev)
        live_end = rdist.reduce_sum(float(live[-1]), dev)
    else:
        live_end = float(live[-1])
    node_ticks = delta["node_ticks"]

    # event model (per launch of one rank's shard): hot state in + out, 64 B per delivered
    # message, 16 B per appended entry (counts are whole-job, divided back to one launch)
    total_launches = max(1, launches * world)
    s_node = 32 + 8 * n
    msgs = delta["delivered"] / total_launches
    entries = delta["entries_appended"] / total_launches
    state_bytes = 2 * s_node * count * n
    event_bytes = state_bytes + 64 * msgs + 16 * entries
    achieved = event_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms else 0.0
    ticks_per_launch = args.steps * TICKS_PER_STEP / max(1, launches)
    window = window_id(spec, args)
    traffic, traffic_src = load_traffic(name, window)
    rec = {
        "value": node_ticks / elapsed_max,
        "unit": "node-ticks/s",
        "ms_per_step": elapsed_max * 1e3 / args.steps,
        "scaling": scaling,
        "window": window,
        "config": {"workload": spec["desc"], "clusters": total, "clusters_per_gpu": count,
                   "nodes": n, "ticks_per_step": TICKS_PER_STEP,
                   "parallelism": f"cluster-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "model": "event: 2*S_node*nodes + 64 B/delivered msg + 16 B/appended entry "
                              "per launch",
                     "bytes_per_launch": event_bytes, "avg_launch_ms": avg_launch_ms,
                     # the hot node state in and out once: what a launch that keeps its messages
                     # on chip (the lane-per-cluster steady kernel) must move through HBM
                     "state_bytes_per_launch": state_bytes,
                     "frac_state_model": state_bytes / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                     if avg_launch_ms else 0.0,
                     "launches": launches, "ticks_per_launch": ticks_per_launch,
                     "kernel_src_sha": kernel_build_hash(),
                     "limiter": LIMITER["c2" if name == "c2" else "c3"]},
        "live_node_frac_end": live_end / (total * n),
        "live_node_ticks_per_s": live_ticks / elapsed_max if dist is None
        else live_ticks / elapsed_max,
        "payload_evicted": delta["payload_evicted"],
        "counters": {k: v for k, v in delta.items() if v},
        "sched_note": "C3 windows sync once per step to count live nodes (counter read ~0.05 ms "
                      "per step, inside the timed region)" if init else None,
    }
    if delta["payload_evicted"]:
        # SIM_SPEC §4 P3: an evicted payload entry is the simulator's one fidelity limit
        rec["fidelity_warning"] = "payload entries were evicted from a sender's arena"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(spec, args)
    sim.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2+c3+c3_spec",
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
            "metric": "simulated node-ticks/sec (5-node Raft)" if WORKLOADS[names[0]]["cfg"]["nodes"] == 5
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
            "window": head["window"],
            "payload_evicted": head["payload_evicted"],
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
