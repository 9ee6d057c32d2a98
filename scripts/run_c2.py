"""Run C2 (65,536 five-node clusters) for a profiler: 3 warm-up launches, then 5 launches.
Usage: run_c2.py LIB [clusters]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

sim = Backend(sys.argv[1], "raft_sim_", n_clusters=int(sys.argv[2]) if len(sys.argv) > 2 else 65536,
              nodes=5, seed=42)
for _ in range(8):
    sim.step(10000)
print("kernel ms", sim.last_step_timing())
