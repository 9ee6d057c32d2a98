"""Per-wave statistics from an RS_WAVESTATS diagnostic build of the tick kernel (build with
-DRS_WAVESTATS): active ticks per wave (mean, max, how many waves exceed 40/60/80/100) and a
wave-level phase clock (s_waitcnt + clock64 at every phase boundary, so the split is of
latency-exposed time, not of the product's overlapped execution). Both land in counters the C2
workload never uses, so the numbers are only meaningful for C2-shaped runs.
Usage: python scripts/wavestats_probe.py LIB"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

lib = sys.argv[1]
for sched, c, q in ((0, 65536, 16), (1, 65536, 16), (0, 16384, 16)):
    if True:
        print(f"== schedule {sched}, {c} clusters, inbox_cap {q}", flush=True)
        sim = Backend(lib, "raft_sim_", n_clusters=c, nodes=5, seed=42, schedule=sched,
                      inbox_cap=q)
        sim.step(10000)
        for step in range(1):
            before = sim.counters()
            sim.step(10000)
            after = sim.counters()
            waves = (c + 11) // 12
            tot = after["payload_evicted"] - before["payload_evicted"]
            print(f"sched {sched} clusters {c} step {step}: kernel {sim.last_step_timing()[0]:.3f} ms, "
                  f"active ticks/wave mean {tot / waves:.1f}, max so far {after['halt_overflow']}, "
                  f"waves >40/60/80/100: " + "/".join(str(after[k] - before[k]) for k in
                  ("halt_npe", "halt_cce", "halt_ioobe", "viol_complete")),
                  flush=True)
            names = ["loop/skip", "P0", "P1 select+pop", "P1 handler", "P1 next/match",
                     "P1 emission", "P2", "P3", "P4", "emit: next loads", "emit: cells"]
            keys = ["dropped", "partitioned", "duplicated", "overflow", "to_halted",
                    "client_injected", "entries_applied", "viol_election", "viol_log", "ev_cs",
                    "entries_appended"]
            cyc = [after[k] - before[k] for k in keys]
            print("   cycles per active tick: " + ", ".join(
                f"{n} {c / max(1, tot):.0f}" for n, c in zip(names, cyc)),
                  flush=True)
        sim.close()
