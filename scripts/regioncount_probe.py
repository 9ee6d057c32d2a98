"""Dynamic code-region profile of one launch from a -DRS_REGIONCOUNT build (diagnostic only): how
many times the waves executed each region of the tick loop (a region counts once per wave pass,
whatever the number of active lanes). Usage: regioncount_probe.py LIB [c2|c3|c4_n9]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "scripts")]
from raftsim._backend import Backend  # noqa: E402
from ab_probe import WORK  # noqa: E402

NAMES = {0: "loop trips", 1: "P0 injection", 2: "P1 entered", 3: "P1 pop", 4: "draw both-ready",
         5: "draw in pop", 6: "draw at re-arm", 7: "timeout/heartbeat", 8: "message switch",
         9: "fault", 10: "no-fault tail", 11: "redirect", 12: "emission", 13: "emit reply",
         14: "emit broadcast", 16: "P2", 17: "P2 insert trips", 19: "P3", 21: "P3 apply",
         22: "P4", 23: "P4 log matching", 25: "drain", 26: "drain trips"}

lib, wl = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "c2")
cfg = dict(WORK[wl])
C, N = cfg["n_clusters"], cfg["nodes"]
sim = Backend(lib, "raft_sim_", **cfg)
for _ in range(4):
    sim.step(10000)
waves = 2 * C // (64 // N) + 1100
buf = (ctypes.c_uint32 * (waves * 32))()
n = sim._lib.raftsim_diag_wavelog(sim._h, buf, waves)
a = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 32)[:n].astype(np.int64)
ran = a[:, 0] > 0
a = a[ran]
print(f"{wl}: kernel {sim.last_step_timing()[0]:.3f} ms, {len(a)} waves with active trips")
tot = a.sum(axis=0)
for i, nm in NAMES.items():
    print(f"  {i:2d} {nm:20s} total {tot[i]:12d}  per wave {tot[i] / len(a):9.2f}")
