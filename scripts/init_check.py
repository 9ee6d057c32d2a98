"""c2_init on a fresh handle (diagnostic): the first 10k-tick step's device span, tick-kernel time,
steady bails, and per-cluster digests of a slice against the C oracle. Usage: init_check.py LIB [C]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
from raftsim._backend import Backend  # noqa: E402

lib = sys.argv[1]
C = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
for rep in range(3):
    s = Backend(lib, "raft_sim_", n_clusters=C, nodes=5, seed=42 + rep)
    s.step_async(10000)
    s.sync()
    ms, nl = s.last_step_timing()
    f = s._lib.raftsim_diag_last_bails
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p]
    print(f"span {s.last_span() * 1e3:7.1f} us  kernel {ms * 1e3:7.1f} us x{nl}  bails {f(s._h)}",
          flush=True)
    if rep == 0:
        import helpers
        r = helpers.oracle(n_clusters=2048, nodes=5, seed=42)
        r.step(10000)
        bad = np.nonzero(s.digest(0, 2048) != r.digest())[0]
        print("digest mismatches in [0, 2048):", len(bad), bad[:8])
    s.close()
