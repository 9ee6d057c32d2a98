"""bench.py — simulated node-ticks/s of the batched Raft simulator on MI355X.

Headline workload (BASELINE.json configs[1], "C2"): 65,536 independent 5-node clusters per GPU, no
faults, no client traffic. One *step* = one raft_sim_step(10,000 ticks) over every cluster,
continuing the simulation; state is resident in HBM before timing starts. Under torchrun each rank
simulates its own 65,536 clusters (global ids rank*65536 + i: disjoint, shard-invariant Philox
streams; weak scaling, no data-path collective). C2 is periodic in steady state (heartbeat rounds
every hb ticks), so its window is the K steps after W warm-up steps.

Timing. Each rank enqueues its K steps on the simulator's stream and syncs once; the device time
of the K steps is taken from HIP events on that stream (raft_sim_last_span: from before the first
launch to after the last), MAX-reduced over ranks, and `value` = all ranks' node-ticks / that
time. The K steps are also bracketed by a barrier + torch.cuda.synchronize() on both sides and the
wall time around them is reported as `wall_ms_per_step` (it adds the host's sync and, under
torchrun, barrier latency, which at C2's ~0.03 ms per step would dominate a 20-step span).

The same JSON line carries, under "workloads", the other BASELINE configs:
  c2_init   config 2 as named: ticks [0, 10,000) from init-node (every cluster elects its first
            leader), on `reps` fresh handles.
  c3        config 3: 1,048,576 five-node clusters with 10 % drop, 1 % duplication, delay U[1,50],
            partitions and a bursty client that follows redirects (SIM_SPEC D14/D15; one
            client-set per 100 ticks on average), ticks [0, 10,000 K) from init-node on a fresh
            handle (the W warm-up steps run on a throwaway handle); under the faithful handlers a
            crash storm, so the line reports the live-node fraction at the window's end.
  c3_spec   the same traffic under the Spec-Raft control (SIM_SPEC §8): real replication at 1M.
  c4_n7,    config 4: 16,384 seven- / nine-node clusters per GPU, 4096-entry logs, bursty client
  c4_n9     (1000+-entry AppendEntries batches, OVERFLOW halts), ticks [0, 10,000 K) from
            init-node like C3 (the replication and the halts are inside the window).
  c4_spec   c4_n9's clusters under the Spec-Raft control: the commit index by the sorting network
            over match_index (tick_wave.hpp).
  c5        config 5: config 3's faults and client with the vote granted without the up-to-date
            check on the Spec-Raft protocol (variant flags 3), 131,072 clusters per GPU, stepped
            1,000 ticks at a time until a safety violation is counted anywhere in the job (a MIN
            all-reduce of the first-violation tick over RCCL per chunk); time to it, and the C
            oracle's time to the same tick on the same clusters.

Per workload:
  roofline      the tick kernel against HBM bandwidth. `achieved` = the compulsory bytes of a
                launch -- the hot node state in and out once, 2 * S_node(N) bytes per node
                (S_node = 32 + 8N) -- over the average launch time measured with HIP
                events on the simulator's stream; `frac` = achieved / 8 TB/s. `traffic` = the
                PMC-measured HBM bytes per launch (pmc_traffic.json, scripts/summarize_profile.py),
                used only when measured on this kernel build (source hash) over this window.
                `frac_event_model` prices SURVEY's event model instead (+ 64 B per delivered
                message + 16 B per appended entry); the steady kernel keeps C2's messages in
                registers, so those bytes never reach HBM there.
  cpu_baseline  the C oracle (oracle/raftref.c, the restatement of core.clj/log.clj; "port") on a
                bounded sample of the same workload over the same tick window, clusters mapped over
                every host CPU this process may run on (the pmap analogue), with the same
                discrete-event idle-tick skipping the GPU kernel does; rank 0 at N=1 only. The
                every-tick restatement's rate is given beside it.
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
from raftsim import _build  # noqa: E402

KERNEL_SOURCES = _build.KERNEL_SOURCES

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
TICKS_PER_STEP = 10000
FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
C3_CFG = dict(nodes=5, seed=1, log_cap=256, client_ppm=80000, client_period=16384,
              client_burst=2048, client_redirects=4, **FAULTS)
C3_DESC = ("1,048,576 five-node clusters across all GPUs x 10,000 ticks per step; drop 10 %, dup 1 "
           "%, delay U[1,50], partitions p=0.1 per 1000-tick epoch; client-sets in bursts (2048 of "
           "every 16384 ticks, 1 per 100 ticks on average) following up to 4 redirects; window: "
           "ticks [0, 10000 * steps) from init-node")
C4_DESC = ("4096-entry logs, bursty client (500,000 ppm in 2048 of every 8192 ticks, up to 4 "
           "redirects followed: 1000+-entry AppendEntries batches, OVERFLOW halts at the cap); "
           "window: ticks [0, 10000 * steps) from init-node")


def C4_CFG(nodes, seed):
    return dict(nodes=nodes, seed=seed, log_cap=4096, client_ppm=500000, client_period=8192,
                client_burst=2048, client_redirects=4)


# name: config, clusters, per-rank scaling, window, CPU sample, description. CPU sample: (clusters,
# steps) after a warm-up step for "steady" windows; for "init" windows cluster-steps, i.e. the
# oracle runs cluster_steps // steps clusters over the GPU's own window from init-node.
WORKLOADS = {
    "c2": dict(short="C2: 65,536 5-node clusters/GPU, 10k ticks/step, no faults, no client (steady window)",
               cfg=dict(nodes=5, seed=42), clusters=65536, scaling="weak", window="steady",
               cpu=(65536, 40),
               desc="C2: 65,536 five-node clusters per GPU x 10,000 ticks per step, no faults, "
                    "no client"),
    "c2_init": dict(short="C2 from init-node: ticks [0,10k), first elections",
                    cfg=dict(nodes=5, seed=42), clusters=65536, scaling="weak", window="first",
                    cpu=65536, reps=5,
                    desc="C2 as named: 65,536 five-node clusters per GPU, ticks [0, 10,000) from "
                         "init-node (first elections included), no faults, no client"),
    "c3": dict(short="C3: 1M 5-node clusters, drop/dup/delay/partitions, bursty redirecting client, [0,10k*K) from init",
               cfg=C3_CFG, clusters=1 << 20, scaling="strong", window="init", cpu=1 << 19,
               desc="C3: " + C3_DESC),
    "c3_spec": dict(short="C3 under Spec-Raft",
                    cfg=dict(C3_CFG, variant_flags=2, log_cap=1024), clusters=1 << 20,
                    scaling="strong", window="init", cpu=1 << 19,
                    desc="C3 under the Spec-Raft control (SIM_SPEC §8, 1024-entry logs): "
                         + C3_DESC),
    # config 4 from init-node, like C3: the window holds the log growth under the bursty client,
    # the 1000+-entry AppendEntries batches (core.clj:56-67 ships the whole suffix, log.clj:61-64)
    # and the OVERFLOW halts at the 4096-entry cap; Spec-Raft is where the commit index comes from
    # the sorting network over match_index
    "c4_n7": dict(short="C4: 16,384 7-node clusters/GPU, 4096-entry logs, bursty client, from init",
                  cfg=C4_CFG(7, 3), clusters=16384, scaling="weak", window="init", cpu=1 << 15,
                  desc="C4: 16,384 seven-node clusters per GPU, " + C4_DESC),
    "c4_n9": dict(short="C4: 16,384 9-node clusters/GPU, 4096-entry logs, bursty client, from init",
                  cfg=C4_CFG(9, 5), clusters=16384, scaling="weak", window="init", cpu=1 << 15,
                  desc="C4: 16,384 nine-node clusters per GPU, " + C4_DESC),
    "c4_spec": dict(short="C4-N9 under Spec-Raft (sorting-network commit)",
                    cfg=dict(C4_CFG(9, 5), variant_flags=2), clusters=16384, scaling="weak",
                    window="init", cpu=1 << 15,
                    desc="C4 under the Spec-Raft control (majority commit index by the sorting "
                         "network over match_index, truncate-on-conflict): 16,384 nine-node "
                         "clusters per GPU, " + C4_DESC),
    "c5": dict(short="C5: 131,072 clusters/GPU, no-log-check vote variant, to first violation",
               cfg=dict(C3_CFG, variant_flags=3, log_cap=1024), clusters=131072, scaling="weak",
               window="violation", chunk=1000, max_ticks=200000,
               desc="C5: 131,072 five-node clusters per GPU with C3's faults and client, Spec-Raft "
                    "with the vote granted without the up-to-date check (variant flags 3); "
                    "stepped 1,000 ticks at a time from init-node until a safety violation is "
                    "counted anywhere in the job"),
}
HALTS = ("halt_ioobe", "halt_npe", "halt_cce", "halt_overflow")
MODEL = {
    "steady": "frac: compulsory bytes (hot state in+out, 2(32+8N) B/node) / launch; frac_measured: "
              "PMC HBM bytes / launch. The 42 MB state stays Infinity-Cache resident between "
              "launches and the launch is dispatch-bound (~3 us empty dispatch + one wave's chain)",
    "general": "frac: compulsory bytes (hot state in+out, 2(32+8N) B/node) / launch; frac_measured: "
               "PMC HBM bytes / launch. Bound by the issue of divergent per-trip instruction "
               "streams, not HBM bandwidth",
}
LIMITER = {
    "steady": "one wave per SIMD running 64 clusters' heartbeat rounds (C2 has exactly 64 clusters "
              "per SIMD): the state load, the chain of dependent multiplies per trip (trace hash; "
              "one Philox draw per follower per launch) and the write-back, in sequence "
              "(per-wave timeline, DESIGN.md); messages stay in registers",
    "general": "issue of the active trips' divergent instruction stream (client-set injections, "
               "redirect hops, replication and checker trips; PMC instruction counts, DESIGN.md), "
               "not HBM bandwidth",
}


def kernel_build_hash():
    """The hash libraftsim.so embeds (raftsim/_build.py): the kernel sources under ROOT."""
    return _build.source_hash(ROOT)


def window_id(spec, args):
    """The tick window a number describes: steady windows are the K steps after W warm-up steps
    (periodic state: any K), init windows ticks [0, 10000 K) from init-node, first windows ticks
    [0, 10000) from init-node, violation windows from init-node to the first violation."""
    if spec["window"] == "init":
        return {"kind": "init", "steps": args.steps}
    if spec["window"] == "first":
        return {"kind": "first", "steps": 1}
    if spec["window"] == "violation":
        return {"kind": "violation", "chunk": spec["chunk"]}
    return {"kind": "steady", "steps": args.steps, "warmup": args.warmup}


def load_traffic(workload, window):
    """PMC HBM bytes per tick-kernel launch measured on THIS kernel source over this window (else
    None, with the reason)."""
    rec, why = load_pmc(workload, window)
    return (rec.get("hbm_bytes_per_launch"), rec.get("source")) if rec else (None, why)


def load_pmc(workload, window):
    """The pmc_traffic.json record of `workload` (HBM bytes, LDS bank conflicts, occupancy per
    tick-kernel launch) if it was measured on THIS kernel source over this window, else (None, the
    reason)."""
    f = ROOT / "pmc_traffic.json"     # written by scripts/summarize_profile.py
    try:
        rec = json.loads(f.read_text()).get(workload)
    except (OSError, ValueError):
        return None, "no pmc_traffic.json"
    if not rec:
        return None, f"no PMC profile of {workload}"
    if rec.get("kernel_src_sha") != kernel_build_hash():
        return None, "PMC profile of another kernel build"
    if rec.get("window") != window:
        return None, f"PMC profile window {rec.get('window')} is not this window"
    return rec, rec.get("source")


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
    elif spec["window"] == "first":
        clusters, steps = spec["cpu"], 1
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
    where = (f"{steps} steps after a warm-up step" if warm
             else f"ticks [0, {steps * TICKS_PER_STEP}) from init-node (the GPU's window)")
    return {"value": v, "unit": "node-ticks/s", "cores": threads, "kind": "port",
            "sample": f"{clusters} clusters x {cfg['nodes']} nodes, {where}, oracle/raftref.c "
                      f"with the same idle-tick skipping as the kernel, {threads} threads (the host "
                      f"CPUs this process may use: affinity mask capped by the cgroup quota), "
                      f"{dt:.2f} s",
            "short_sample": f"{clusters} clusters, {where}, oracle/raftref.c, {threads} threads",
            "host_cpus": hc,
            "every_tick_value": v_every,
            "every_tick_sample": f"{max(1, clusters // 8)} clusters x 1 step visiting every tick, "
                                 f"{dt_every:.2f} s"}


def roofline(name, spec, count, n, launches, avg_launch_ms, delta, window, world,
             launch_src="HIP events in the launches' dispatch packets, averaged over the timed "
                        "launches"):
    """Compulsory-byte roofline of the dominant kernel (per launch of one rank's shard)."""
    total_launches = max(1, launches * world)
    s_node = 32 + 8 * n
    msgs = delta["delivered"] / total_launches
    entries = delta["entries_appended"] / total_launches
    state_bytes = 2 * s_node * count * n
    event_bytes = state_bytes + 64 * msgs + 16 * entries
    gbs = (lambda b: b / (avg_launch_ms * 1e-3) / 1e9) if avg_launch_ms else (lambda b: 0.0)
    pmc, traffic_src = load_pmc(name, window)
    pmc = pmc or {}
    traffic = pmc.get("hbm_bytes_per_launch")
    steady = spec["cfg"]["nodes"] <= 5 and not spec["cfg"].get("client_ppm") and \
        spec["window"] in ("steady",)
    return {"bound": "hbm", "achieved": gbs(state_bytes), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs(state_bytes) / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": traffic_src,
            # the PMC-measured bytes over the same launch time: what the memory system moved
            "frac_measured": gbs(traffic) / HBM_PEAK_GBS if traffic else None,
            "lds_bank_conflict_per_lds_inst": pmc.get("lds_bank_conflict_per_lds_inst"),
            "waves_per_simd": pmc.get("waves_per_simd"),
            "valu_insts_per_wave": pmc.get("valu_insts_per_wave"),
            "model": MODEL["steady" if steady else "general"],
            "bytes_per_launch": state_bytes, "avg_launch_ms": avg_launch_ms,
            "avg_launch_source": launch_src,
            "traffic_over_compulsory": traffic / state_bytes if traffic else None,
            "frac_event_model": gbs(event_bytes) / HBM_PEAK_GBS,
            "event_bytes_per_launch": event_bytes,
            "launches": launches, "kernel_src_sha": kernel_build_hash(),
            "limiter": LIMITER["steady" if steady else "general"]}


def survey_8d(rate, n, delta):
    """SURVEY §8(d)'s per-node-tick accounting, B(N) = 2(32 + 8N) + 8 + 64 m + 16 e bytes per
    simulated node-tick, priced at the line's rate: a 'fraction' above 1 means the kernels never
    touch most node-ticks (idle ticks are skipped exactly, fixed-point rounds fold into hashes),
    so it measures the algorithm, not the memory system; `frac` (compulsory bytes per launch over
    the launch time) is the physical fraction."""
    nt = max(1, delta["node_ticks"])
    b = 2 * (32 + 8 * n) + 8 + 64 * delta["delivered"] / nt + 16 * delta["entries_appended"] / nt
    return {"bytes_per_node_tick": b, "value": rate * b / (HBM_PEAK_GBS * 1e9),
            "note": "SURVEY 8(d) rate x B / 8e12; not a bandwidth fraction here (idle node-ticks "
                    "are skipped exactly, so it exceeds 1): see frac"}


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
    dev = f"cuda:{local_rank}"

    def make():
        return raftsim.Simulator(n_clusters=count, cluster_offset=offset, device=local_rank, **cfg)

    def barrier():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    window = window_id(spec, args)
    kind = spec["window"]
    extra = {}
    if kind == "violation":
        return run_violation(name, spec, args, world, rank, dist, make, count, total, offset)
    if kind == "init" and args.warmup:       # same shape, thrown away: the window starts at init
        w = make()
        for _ in range(args.warmup):
            w.step(TICKS_PER_STEP)
        w.sync()
        w.close()
    # config 2 as named: a fresh handle per repetition, created (alloc + init-node kernel) before
    # the timed region; each repetition is one 10k-tick step from init-node
    sims = [make() for _ in range(spec["reps"])] if kind == "first" else [make()]
    sim = sims[0] if kind != "first" else None
    if kind == "steady":
        for _ in range(args.warmup):
            sim.step(TICKS_PER_STEP)
    nodes = count * n
    c_before = sim.counters() if sim else None
    live = [nodes - sum(c_before[h] for h in HALTS)] if sim else []
    steps = args.steps if kind != "first" else 1
    barrier()
    t0 = time.perf_counter()
    span_ms, kernel_ms, launches = 0.0, 0.0, 0
    if kind == "first":
        c_sum = None
        for s in sims:
            s.step_async(TICKS_PER_STEP)
            s.sync()
        wall_first = time.perf_counter() - t0
        for s in sims:
            span_ms += s.last_span()
            ms, nl = s.last_step_timing()
            kernel_ms += ms * nl
            launches += nl
            c = s.counters()
            c_sum = c if c_sum is None else {k: (c_sum[k] + c[k]) if isinstance(c[k], int) and
                                             k not in ("first_violation_tick", "payload_max")
                                             else c[k] for k in c}
        steps = len(sims)
    elif kind == "init":
        # one sync per step: the live-node count after every step (halts are permanent, so the
        # halt counters count the halted nodes); the device time of each step is its own span
        for _ in range(steps):
            sim.step_async(TICKS_PER_STEP)
            sim.sync()
            span_ms += sim.last_span()
            ms, nl = sim.last_step_timing()
            kernel_ms += ms * nl
            launches += nl
            c = sim.counters()
            live.append(nodes - sum(c[h] for h in HALTS))
    else:
        # K steps enqueued back to back on the simulator's stream (raft_sim_step_async), then one
        # raft_sim_sync: HIP events time the whole span and every tick-kernel launch in it
        for _ in range(steps):
            sim.step_async(TICKS_PER_STEP)
        sim.sync()
        span_ms = sim.last_span()
        ms, launches = sim.last_step_timing()
        kernel_ms = ms * launches
    barrier()
    wall = time.perf_counter() - t0
    if kind == "first":
        wall = wall_first          # the counter reads after the steps are not the steps' time
    avg_launch_ms = kernel_ms / max(1, launches)
    timed = sim.timed_launches() if sim is not None else launches
    launch_src = (f"HIP events in the launches' dispatch packets, averaged over the {timed} timed "
                  f"launches")
    if kind == "steady" and steps:
        # A steady window is one dispatch per step, and only the first launch after the sync
        # carries events (an event pair costs ~6 us per dispatch): one timed launch is a sample of
        # one, so the roofline takes the device span per step, which bounds the average launch
        # from above (it adds the gaps between back-to-back launches)
        extra["timed_launch_ms"] = avg_launch_ms
        extra["timed_launches"] = timed
        avg_launch_ms = span_ms / steps
        launch_src = ("device span / steps: one dispatch per step, so this bounds the average "
                      f"launch from above (the {timed} event-timed launch: timed_launch_ms)")
    if kind == "first":
        delta = {k: v for k, v in c_sum.items()}
        live = [nodes, nodes - sum(c_sum[h] for h in HALTS) // max(1, spec["reps"])]
    else:
        c_after = sim.counters()
        if kind == "steady":
            live.append(nodes - sum(c_after[h] for h in HALTS))
        delta = {k: c_after[k] - c_before[k] for k in c_after
                 if k not in ("first_violation_tick", "payload_max")}
        delta["payload_max"] = c_after["payload_max"]
        delta["first_violation_tick"] = c_after["first_violation_tick"]
    live_ticks = (sum((a + b) / 2 for a, b in zip(live, live[1:])) * TICKS_PER_STEP
                  if kind == "init" else (live[0] + live[-1]) / 2 * TICKS_PER_STEP * steps)
    span_max, wall_max = span_ms, wall
    if dist is not None:
        span_max = rdist.reduce_max(span_ms, dev)
        wall_max = rdist.reduce_max(wall, dev)
        delta = rdist.reduce_counters(delta, dev)
        avg_launch_ms = rdist.reduce_max(avg_launch_ms, dev)
        live_ticks = rdist.reduce_sum(live_ticks, dev)
        live_end = rdist.reduce_sum(float(live[-1]), dev)
    else:
        live_end = float(live[-1])
    node_ticks = delta["node_ticks"]
    rec = {
        "value": node_ticks / (span_max * 1e-3),
        "unit": "node-ticks/s",
        "ms_per_step": span_max / steps,
        "wall_ms_per_step": wall_max * 1e3 / steps,
        "wall_value": node_ticks / wall_max,
        "timing": "device time of the steps (HIP events on the simulator's stream, MAX over "
                  "ranks); wall_* = perf_counter around them, barrier + synchronize both sides",
        "scaling": scaling,
        "window": window,
        "config": {"workload": spec["desc"], "clusters": total, "clusters_per_gpu": count,
                   "nodes": n, "ticks_per_step": TICKS_PER_STEP,
                   "parallelism": f"cluster-sharded x{world}"},
        "roofline": roofline(name, spec, count, n, launches, avg_launch_ms, delta, window, world,
                             launch_src),
        "events_per_s": sum(delta[k] for k in delta if k.startswith("ev_")) / (span_max * 1e-3),
        "live_node_frac_end": live_end / (total * n),
        "live_node_ticks_per_s": live_ticks / (span_max * 1e-3),
        "payload_evicted": delta["payload_evicted"],
        "ev_ae": delta["ev_ae"],
        "payload_max": delta["payload_max"],
        "counters": {k: v for k, v in delta.items() if v},
        **extra,
    }
    rec["roofline"]["survey_8d"] = survey_8d(rec["value"], n, delta)
    if kind == "first":
        rec["reps"] = spec["reps"]
    if delta["payload_evicted"]:
        # SIM_SPEC §4 P3: an evicted payload entry is the simulator's one fidelity limit
        rec["fidelity_warning"] = "payload entries were evicted from a sender's arena"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(spec, args)
    for s in sims:
        s.close()
    return rec


def run_violation(name, spec, args, world, rank, dist, make, count, total, offset):
    """BASELINE config 5: step every rank's clusters chunk by chunk until a violation is counted
    anywhere in the job (MIN all-reduce of the first-violation tick per chunk over RCCL)."""
    from raftsim import dist as rdist

    cfg, n = spec["cfg"], spec["cfg"]["nodes"]
    dev = f"cuda:{os.environ.get('LOCAL_RANK', '0')}"
    red = (lambda x: rdist.reduce_min(x, dev)) if dist is not None else None
    sim = make()
    t0 = time.perf_counter()
    fv, ticks, (span_ms, kms, launches) = rdist.first_violation_search(
        sim, spec["chunk"], spec["max_ticks"], red)
    wall = time.perf_counter() - t0
    avg_launch_ms = kms / max(1, launches)
    c = sim.counters()
    span_max = span_ms
    if dist is not None:
        span_max = rdist.reduce_max(span_ms, dev)
        avg_launch_ms = rdist.reduce_max(avg_launch_ms, dev)
        c = rdist.reduce_counters(c, dev)
    window = window_id(spec, args)
    rec = {
        "value": c["node_ticks"] / (span_max * 1e-3),
        "unit": "node-ticks/s",
        "first_violation_tick": fv,
        "ticks_simulated": ticks,
        "time_to_first_violation_s": span_max * 1e-3,
        "ms_per_step": span_max / max(1, ticks // spec["chunk"]),     # per chunk of ticks
        "wall_s": wall,
        "timing": "device time of the chunks (HIP events, MAX over ranks); wall_s adds the "
                  "per-chunk counter reads and all-reduces",
        "scaling": "weak",
        "window": window,
        "config": {"workload": spec["desc"], "clusters": total, "clusters_per_gpu": count,
                   "nodes": n, "ticks_per_chunk": spec["chunk"],
                   "parallelism": f"cluster-sharded x{world}"},
        "roofline": roofline(name, spec, count, n, launches, avg_launch_ms, c, window, world),
        "counters": {k: v for k, v in c.items() if v},
    }
    rec["roofline"]["survey_8d"] = survey_8d(rec["value"], n, c)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import helpers

        ref = helpers.oracle(n_clusters=count, cluster_offset=offset, **cfg)
        threads = helpers.cpu_threads()
        helpers.oracle_threads(ref, threads)
        helpers.oracle_idle_skip(ref, True)
        t1 = time.perf_counter()
        cfv, cticks, _ = rdist.first_violation_search(ref, spec["chunk"], ticks)
        dt = time.perf_counter() - t1
        rec["cpu_baseline"] = {
            "value": count * n * cticks / dt, "unit": "node-ticks/s", "cores": threads,
            "kind": "port", "time_to_first_violation_s": dt, "first_violation_tick": cfv,
            "bit_exact": cfv == fv and cticks == ticks and bool((sim.digest() == ref.digest()).all()),
            "sample": f"the same {count} clusters x {n} nodes from init-node in the same "
                      f"{spec['chunk']}-tick chunks, oracle/raftref.c with idle-tick skipping, "
                      f"{threads} threads, {dt:.2f} s",
            "host_cpus": host_cpus()}
    sim.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2+c2_init+c3+c3_spec+c4_n7+c4_n9+c4_spec+c5",
                    help="headline[+extra...] from " + ", ".join(WORKLOADS))
    ap.add_argument("--clusters", type=int, default=0, help="override the headline's clusters")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--full-json", default=None,
                    help="where the full per-workload records go (default gpurun_out/bench_full.json)")
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
        full = args.full_json or str(ROOT / "gpurun_out" / "bench_full.json")
        try:
            Path(full).parent.mkdir(parents=True, exist_ok=True)
            Path(full).write_text(json.dumps({"n_gpus": world, "steps": args.steps,
                                              "warmup": args.warmup, "workloads": recs},
                                             indent=1) + "\n")
        except OSError as e:                      # the full record is a convenience; the line is not
            print(f"bench: could not write {full}: {e}", file=sys.stderr)
            full = None
        print(json.dumps(compact_line(names, recs, world, args, full)), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _r(x, d=4):
    """Round for the line: floats to d significant digits (the driver keeps ~8 KB of stdout)."""
    if isinstance(x, float):
        return float(f"{x:.{d}g}")
    return x


ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "frac_measured", "traffic",
             "traffic_over_compulsory", "bytes_per_launch", "avg_launch_ms",
             "lds_bank_conflict_per_lds_inst", "waves_per_simd")
WL_KEYS = ("value", "ms_per_step", "live_node_frac_end", "ev_ae", "payload_max",
           "first_violation_tick", "time_to_first_violation_s")


def compact_line(names, recs, world, args, full_path):
    """The ONE JSON line bench.py prints: the headline workload's keys, its roofline and CPU
    baseline, and per workload only its rate, step time, roofline fractions and traffic, CPU rate
    and the fields that say what the window held; the full records go to `full_path`. Kept well
    under 8,000 characters (tests/test_bench_contract.py)."""
    head = recs[names[0]]
    n = WORKLOADS[names[0]]["cfg"]["nodes"]
    out = {
        "metric": "simulated node-ticks/sec (5-node Raft)" if n == 5 else "simulated node-ticks/sec",
        "value": _r(head["value"], 6),
        "unit": "node-ticks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": _r(head["ms_per_step"], 6),
        "higher_is_better": True,
        "scaling": head["scaling"],
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded Philox clusters from init-node state)",
        "config": {"workload": WORKLOADS[names[0]]["short"],
                   **{k: head["config"][k] for k in ("clusters", "clusters_per_gpu", "nodes",
                                                      "parallelism")}},
        "roofline": {k: _r(head["roofline"].get(k)) for k in ROOF_KEYS},
        "wall_ms_per_step": _r(head.get("wall_ms_per_step")),
        "events_per_s": _r(head.get("events_per_s")),
    }
    out["roofline"]["model"] = head["roofline"]["model"]
    if "timed_launch_ms" in head:
        out["timed_launch_ms"] = _r(head["timed_launch_ms"])
    cb = head.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {"value": _r(cb["value"]), "unit": cb["unit"], "cores": cb["cores"],
                               "kind": cb["kind"], "sample": cb.get("short_sample", cb["sample"])}
    wls = {}
    for name in names[1:]:
        r = recs[name]
        w = {k: _r(r[k]) for k in WL_KEYS if k in r}
        roof = r["roofline"]
        for k in ("frac", "frac_measured", "traffic", "lds_bank_conflict_per_lds_inst",
                  "waves_per_simd"):
            w[k] = _r(roof.get(k))
        if "cpu_baseline" in r:
            w["cpu"] = _r(r["cpu_baseline"]["value"])
            if "bit_exact" in r["cpu_baseline"]:
                w["cpu_bit_exact"] = r["cpu_baseline"]["bit_exact"]
        wls[name] = w
    if wls:
        out["workloads"] = wls
    out["full_record"] = os.path.relpath(full_path, ROOT) if full_path else None
    return out


if __name__ == "__main__":
    main()
