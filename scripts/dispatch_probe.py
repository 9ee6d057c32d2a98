"""Device time per C2 step of the library builds given (diagnostic): the normal build and probe
builds (e.g. -DRS_WAVELOG, built by scripts/build_variants.sh). Usage:
dispatch_probe.py LIB [LIB ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

for lib in sys.argv[1:]:
    for rep in range(3):
        sim = Backend(lib, "raft_sim_", n_clusters=65536, nodes=5, seed=42)
        for _ in range(3):
            sim.step(10000)
        for _ in range(20):
            sim.step_async(10000)
        sim.sync()
        ms, n = sim.last_step_timing()
        print(f"{Path(lib).name:28s} step {sim.last_span() / 20 * 1e3:7.2f} us  launch {ms * 1e3:7.2f} us",
              flush=True)
        sim.close()
