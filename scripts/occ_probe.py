"""Occupancy probe: C2 tick-kernel time vs cluster count, per build (one GPU call). A step in time
at multiples of the resident-wave capacity shows the launch running in generations; the time at
1,024 waves (one per SIMD) is one wave's own latency.
Usage: occ_probe.py LIB [LIB ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

libs = sys.argv[1:] or [str(ROOT / "raft-simulation_amd/build/libraftsim.so")]
for c in [12288, 24576, 36864, 49152, 61440, 65536, 98304]:
    for lib in libs:
        sim = Backend(lib, "raft_sim_", n_clusters=c, nodes=5, seed=42)
        for _ in range(3):
            sim.step(10000)
        ms = []
        for _ in range(4):
            sim.step(10000)
            ms.append(sim.last_step_timing()[0])
        sim.close()
        ms.sort()
        print(f"{Path(lib).name:24s} clusters {c:7d} waves {(c + 11) // 12:6d} kernel median "
              f"{(ms[1] + ms[2]) / 2:7.4f} ms min {ms[0]:7.4f}", flush=True)
