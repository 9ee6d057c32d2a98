"""Wave-packing A/B (one GPU call): each workload run with RAFT_SCHED_ALIGNED (0) and
RAFT_SCHED_FIXED (1) in one process, interleaved; prints median/min ms per 10k-tick step (the
step includes the key + radix-sort kernels of the aligned schedule) and whether the two runs agree
on every cluster digest and counter."""
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
import raftsim  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
WORK = {
    "c2": dict(n_clusters=65536, nodes=5, seed=42),
    "c3": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=10000, log_cap=256, **FAULTS),
    "c3_noclient": dict(n_clusters=131072, nodes=5, seed=1, log_cap=256, **FAULTS),
    "c4_n9": dict(n_clusters=16384, nodes=9, seed=5, client_ppm=250000, log_cap=4096),
}


def main():
    names = sys.argv[1:] or list(WORK)
    for name in names:
        sims = [raftsim.Simulator(**WORK[name], schedule=s) for s in (0, 1)]
        times = [[], []]
        for r in range(6):
            for i, s in enumerate(sims):
                wall = s.step(10000)
                if r:
                    times[i].append(s.last_step_timing()[0])
        same = (np.array_equal(sims[0].digest(), sims[1].digest())
                and sims[0].counters() == sims[1].counters())
        for lbl, ts in zip(("aligned", "fixed"), times):
            print(f"{name:12s} {lbl:8s} median {statistics.median(ts):8.3f} ms  min {min(ts):8.3f} ms",
                  flush=True)
        print(f"{name:12s} identical results: {same}", flush=True)
        for s in sims:
            s.close()


if __name__ == "__main__":
    main()
