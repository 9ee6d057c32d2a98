"""C2 tick-kernel time vs the queue/arena footprint (inbox_cap, log_cap) at the same dynamics: C2
never queues more than N-1 messages per node nor appends an entry, so Q >= 4 and any L give
identical results; only the bytes the queues and arenas span change (TLB / cache reach)."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
import raftsim  # noqa: E402

CASES = [(16, 64), (4, 64), (16, 4), (4, 4), (8, 8)]
sims = {qc: raftsim.Simulator(n_clusters=65536, nodes=5, seed=42, inbox_cap=qc[0], log_cap=qc[1])
        for qc in CASES}
for s in sims.values():
    s.step(10000)
times = {qc: [] for qc in CASES}
for _ in range(6):
    for qc, s in sims.items():
        s.step(10000)
        times[qc].append(s.last_step_timing()[0])
ref = None
for qc, s in sims.items():
    d = bytes(s.digest(0, 512))
    ref = ref or d
    print(f"inbox_cap {qc[0]:2d} log_cap {qc[1]:3d}: kernel median {statistics.median(times[qc]):.3f} ms "
          f"min {min(times[qc]):.3f} ms  same state: {d == ref}", flush=True)
