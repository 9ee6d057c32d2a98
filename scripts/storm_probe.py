"""First launches of a workload with the storm ticks on the lane-per-cluster storm kernel or on the
lane-per-node STORM body (diagnostic): launch times, the storm kernel's leftover count, and whether
both paths give the same state. Usage: python scripts/storm_probe.py WORKLOAD CLUSTERS"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT)]
import bench  # noqa: E402
import raftsim  # noqa: E402

wl, c = sys.argv[1], int(sys.argv[2])
cfg = bench.WORKLOADS[wl]["cfg"]
digests = []
for mode in ("body", "kernel"):
    os.environ["RAFTSIM_STORM_MIN_CLUSTERS"] = "4000000000" if mode == "body" else "1"
    sim = raftsim.Simulator(n_clusters=c, **cfg)
    for i in range(3):
        sim.step(10000)
        ms, nl = sim.last_step_timing()
        print(f"{wl} {c} storm-{mode:6s} step {i} launches {nl} avg ms {ms:.3f} span ms "
              f"{sim.last_span():.3f} storm bails {sim.diag_storm_bails()}", flush=True)
    digests.append(sim.digest())
    sim.close()
print("same state:", bool((digests[0] == digests[1]).all()))
