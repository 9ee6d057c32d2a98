"""Per-launch kernel time of a workload's first launches at several cluster counts (diagnostic):
whether the general kernel is bound by its waves' dependent chains (time flat in the cluster
count while the chip has room) or by issue (time proportional to it).
Usage: python scripts/scale_probe.py WORKLOAD C1 C2 ...   (WORKLOAD a bench.py name)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT)]
import bench  # noqa: E402
import raftsim  # noqa: E402

wl = sys.argv[1]
cfg = bench.WORKLOADS[wl]["cfg"]
for c in map(int, sys.argv[2:]):
    sim = raftsim.Simulator(n_clusters=c, **cfg)
    ms = []
    for _ in range(6):
        sim.step(10000)
        ms.append(sim.last_step_timing()[0])
    print(f"{wl} clusters {c:7d} launch ms " + " ".join(f"{x:7.3f}" for x in ms), flush=True)
    sim.close()
