"""Occupancy probe: C2 kernel time vs cluster count (one GPU call). A step in time at multiples
of the resident-wave capacity shows the launch running in rounds."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
import raftsim  # noqa: E402

for c in [int(x) for x in sys.argv[1:]] or [12288, 24576, 36864, 49152, 53248, 61440, 65536, 98304]:
    sim = raftsim.Simulator(n_clusters=c, nodes=5, seed=42)
    sim.step(10000)
    sim.step(10000)
    ms, n = sim.last_step_timing()
    waves = (c + 11) // 12
    print(f"clusters {c:7d} waves {waves:6d} kernel {ms:7.3f} ms  {c * 5e4 / ms / 1e9 * 1e3:.3e} node-ticks/s",
          flush=True)
