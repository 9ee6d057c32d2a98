"""Quick throughput probe over several configs (one GPU call). Prints one line per config."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

import raftsim  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
PROBES = {
    "idle": dict(n_clusters=65536, nodes=5, el_base=10 ** 8),
    "c2": dict(n_clusters=65536, nodes=5, seed=42),
    "c2_q4": dict(n_clusters=65536, nodes=5, seed=42, inbox_cap=4),
    "c3": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=10000, log_cap=256, **FAULTS),
    "c3_lowclient": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=200, log_cap=256, **FAULTS),
    "c2_client1": dict(n_clusters=65536, nodes=5, seed=42, client_ppm=1),
    "c3_noclient": dict(n_clusters=131072, nodes=5, seed=1, log_cap=256, **FAULTS),
    "c4_n9": dict(n_clusters=16384, nodes=9, seed=5, client_ppm=250000, log_cap=4096),
}


def main():
    check = "--check" in sys.argv
    names = [a for a in sys.argv[1:] if a != "--check"] or list(PROBES)
    for name in names:
        cfg = PROBES[name]
        sim = raftsim.Simulator(**cfg)
        sim.step(10000)
        t0 = time.perf_counter()
        sim.step(10000)
        sim.step(10000)
        dt = (time.perf_counter() - t0) / 2
        ms, n = sim.last_step_timing()
        nt = cfg["n_clusters"] * cfg["nodes"] * 10000
        c = sim.counters()
        ev = sum(c[k] for k in c if k.startswith("ev_")) / max(1, c["node_ticks"])
        print(f"{name:14s} wall {dt*1e3:8.2f} ms/10k ticks  kernel {ms:8.2f} ms  "
              f"{nt/dt:.3e} node-ticks/s  events/node-tick {ev:.2e}", flush=True)
    if check:
        import helpers
        cfg = dict(n_clusters=2048, nodes=5, seed=1, client_ppm=1000, log_cap=256, **FAULTS)
        g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
        helpers.oracle_threads(r, helpers.cpu_threads())
        g.step(20000)
        r.step(20000)
        ok = np.array_equal(g.digest(), r.digest()) and g.counters() == r.counters()
        print("parity check:", "OK" if ok else "MISMATCH", flush=True)


if __name__ == "__main__":
    main()
