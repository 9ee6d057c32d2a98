"""One launch of a bench workload from init-node (ticks [0, 10k)), for PMC passes (diagnostic).
Usage: first_launch.py WORKLOAD CLUSTERS STEPS LIB"""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

spec = importlib.util.spec_from_file_location("bench_cfg", ROOT / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
wl, C, K, lib = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
sim = Backend(lib, "raft_sim_", n_clusters=C, **bench.WORKLOADS[wl]["cfg"])
for _ in range(K):
    sim.step(10000)
    ms, nl = sim.last_step_timing()
    print(f"{wl} launch ms {sim.last_span():.3f} (step span; {nl} launches, avg {ms:.3f})",
          flush=True)
sim.close()
