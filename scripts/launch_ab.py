"""Per-launch kernel time of several builds over the same window from init-node, launch by launch
in one process (cdna_hip_programming.md §5.4 rule 24), and whether their states agree.
Usage: python scripts/launch_ab.py LIB_A LIB_B ... --c4_n9 [--c4_n7 ...] (workloads of ab_probe.py)"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "scripts")]
from raftsim._backend import Backend  # noqa: E402
from ab_probe import WORK  # noqa: E402

libs = [a for a in sys.argv[1:] if not a.startswith("--")]
only = [a[2:] for a in sys.argv[1:] if a.startswith("--")]
for wname in only:
    cfg = WORK[wname]
    sims = [Backend(lib, "raft_sim_", **cfg) for lib in libs]
    tot = [0.0] * len(libs)
    for step in range(20):
        row = []
        for i, s in enumerate(sims):
            s.step(10000)
            ms = s.last_step_timing()[0]
            tot[i] += ms
            row.append(f"{ms:8.3f}")
        print(f"{wname} launch {step:2d} " + " ".join(row), flush=True)
    print(f"{wname} total " + " ".join(f"{x:8.2f}" for x in tot), flush=True)
    d = {bytes(s.digest(0, 2048)) for s in sims}
    print(f"{wname} agree {len(d) == 1}", flush=True)
    for s in sims:
        s.close()
