"""Per-launch burst-engine diagnostics of a -DRS_BURST_DIAG=1 build (tick_wave.hpp; wrong counters,
timing only): engine ticks, engine entries, yields and tick-loop trips per launch.
Usage: python scripts/burst_diag.py LIB c4_n9 [c4_n7 ...]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "scripts")]
from raftsim._backend import Backend  # noqa: E402
from ab_probe import WORK  # noqa: E402

lib = sys.argv[1]
for wname in sys.argv[2:]:
    s = Backend(lib, "raft_sim_", **WORK[wname])
    prev = None
    for step in range(20):
        s.step(10000)
        c = s.counters()
        cur = {k: c[k] for k in ("dropped", "duplicated", "partitioned", "payload_evicted", "ev_cs")}
        d = {k: cur[k] - (prev[k] if prev else 0) for k in cur}
        prev = cur
        print(f"{wname} launch {step:2d} {s.last_step_timing()[0]:8.3f} ms  engine_ticks {d['dropped']:9d} "
              f"entries {d['duplicated']:8d} yields {d['partitioned']:8d} trips {d['payload_evicted']:9d} "
              f"ev_cs {d['ev_cs']:9d}", flush=True)
    s.close()
