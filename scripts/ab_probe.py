"""A/B kernel builds in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
Usage: python scripts/ab_probe.py LIB_A LIB_B ... [--sched=0|1] [--WORKLOAD ...]; prints the median and min kernel ms per
10k-tick launch for each build on each workload, and whether the builds agree on the state."""
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
BURSTS = dict(client_period=16384, client_burst=2048, client_redirects=4)
WORK = {
    "c2": dict(n_clusters=65536, nodes=5, seed=42),
    "c3": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=80000, log_cap=256, **BURSTS,
               **FAULTS),
    "c4_n9": dict(n_clusters=16384, nodes=9, seed=5, client_ppm=500000, log_cap=4096,
                  client_period=8192, client_burst=2048, client_redirects=4),
    "c4_n7": dict(n_clusters=16384, nodes=7, seed=3, client_ppm=500000, log_cap=4096,
                  client_period=8192, client_burst=2048, client_redirects=4),
    "c4_spec": dict(n_clusters=16384, nodes=9, seed=5, client_ppm=500000, log_cap=4096,
                    client_period=8192, client_burst=2048, client_redirects=4, variant_flags=2),
    "c3_spec": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=80000, log_cap=1024, **BURSTS,
                    **FAULTS, variant_flags=2),
}


def main():
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    sched = [int(a[8:]) for a in sys.argv[1:] if a.startswith("--sched=")]
    only = [a[2:] for a in sys.argv[1:]
            if a.startswith("--") and not a.startswith(("--sched=", "--rounds="))]
    extra = {"schedule": sched[0]} if sched else {}
    rounds = 5
    rr = [int(a[9:]) for a in sys.argv[1:] if a.startswith("--rounds=")]
    rounds = rr[0] if rr else rounds
    for wname, cfg in WORK.items():
        if only and wname not in only:
            continue
        sims = [Backend(lib, "raft_sim_", **cfg, **extra) for lib in libs]
        for s in sims:
            s.step(10000)                               # warm up to a steady state
        times = [[] for _ in libs]
        walls = [[] for _ in libs]
        for _ in range(rounds):
            for i, s in enumerate(sims):
                t0 = time.perf_counter()
                s.step(10000)
                walls[i].append((time.perf_counter() - t0) * 1e3)
                times[i].append(s.last_step_timing()[0])
        digests = {bytes(s.digest(0, 256)) for s in sims}
        for lib, ts, ws in zip(libs, times, walls):
            print(f"{wname:6s} {Path(lib).name:28s} median {statistics.median(ts):8.3f} ms  "
                  f"min {min(ts):8.3f} ms  sum {sum(ts):9.3f} ms  step wall median "
                  f"{statistics.median(ws):8.3f} ms", flush=True)
        print(f"{wname:6s} builds agree on state: {len(digests) == 1}", flush=True)
        for s in sims:
            s.close()


if __name__ == "__main__":
    main()
