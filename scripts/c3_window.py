"""C3 from init-node, per-launch tick-kernel time over a window, per build (diagnostic).
Usage: [SPEC=1] c3_window.py CLUSTERS STEPS LIB [LIB ...]   (SPEC=1: the C3-spec workload)"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

C, K = int(sys.argv[1]), int(sys.argv[2])
CFG = dict(nodes=5, seed=1, log_cap=256, client_ppm=80000, client_period=16384, client_burst=2048,
           client_redirects=4, drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
if os.environ.get("SPEC") == "1":
    CFG.update(variant_flags=2, log_cap=1024)
res = {}
for lib in sys.argv[3:]:
    sim = Backend(lib, "raft_sim_", n_clusters=C, **CFG)
    ms = []
    for _ in range(K):
        sim.step(10000)
        ms.append(sim.last_step_timing()[0])
    d = sim.digest(0, min(C, 512))
    sim.close()
    res[lib] = (ms, bytes(d))
    print(f"{Path(lib).name:26s} total {sum(ms):8.2f} ms  per launch " +
          " ".join(f"{m:.2f}" for m in ms), flush=True)
print("builds agree:", len({v[1] for v in res.values()}) == 1)
