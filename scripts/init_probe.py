"""c2_init probe (diagnostic): the first 10k-tick launch of fresh 65,536-cluster handles under both
packing modes (RAFT_SCHED_ALIGNED = 0, RAFT_SCHED_FIXED = 1): device span of the step (HIP events,
packing kernels included) and the tick kernel's own time. Usage: init_probe.py [LIB]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "raft-simulation_amd/build/libraftsim.so")
for rep in range(3):
    for sched in (0, 1):
        sims = [Backend(lib, "raft_sim_", n_clusters=65536, nodes=5, seed=42 + i, schedule=sched)
                for i in range(3)]
        for s in sims:
            s.step_async(10000)
            s.sync()
            ms, nl = s.last_step_timing()
            print(f"sched {sched} span {s.last_span() * 1e3:8.1f} us  tick kernel {ms * 1e3:8.1f} us "
                  f"x{nl}", flush=True)
            s.close()
