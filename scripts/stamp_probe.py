"""Where an active tick spends its cycles: runs an RS_STAMPS diagnostic build of the tick kernel
(see tick_kernel.hip) and prints each phase's share of the wave-cycles, summed over waves.
Usage: python scripts/stamp_probe.py LIB [workload ...]. Shares only; the build's times are not
the product's (every stamp drains the LDS queue)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
WORK = {
    "c2": dict(n_clusters=65536, nodes=5, seed=42),
    "c3": dict(n_clusters=131072, nodes=5, seed=1, client_ppm=10000, log_cap=256, **FAULTS),
    "c4_n9": dict(n_clusters=16384, nodes=9, seed=5, client_ppm=250000, log_cap=4096),
}
PHASES = ["loop+tail", "P0 inject", "P1 event", "P2 deliver", "P3 logs", "P4 checker",
          "next-event"]


def main():
    lib = sys.argv[1]
    for name in sys.argv[2:] or list(WORK):
        cfg = WORK[name]
        sim = Backend(lib, "raft_sim_", **cfg)
        sim.step(20000)
        n = (cfg["n_clusters"] + 63) * 8
        buf = np.zeros(n, dtype=np.uint64)
        f = sim._lib.raft_sim_debug_stamps
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]
        got = f(sim._h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        st = buf[:got].reshape(-1, 8)
        st = st[st[:, 7] > 0]
        tot = st[:, :7].sum()
        ticks = st[:, 7].sum()
        print(f"{name}: {len(st)} waves, {ticks / len(st):.0f} active ticks per wave per 20k ticks, "
              f"{tot / ticks:.0f} cycles per active tick", flush=True)
        for i, ph in enumerate(PHASES):
            print(f"   {ph:12s} {100.0 * st[:, i].sum() / tot:5.1f} %  "
                  f"{st[:, i].sum() / ticks:8.0f} cyc/active tick", flush=True)
        sim.close()


if __name__ == "__main__":
    main()
