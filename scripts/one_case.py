"""Run one GPU parity case of tests/test_gpu_parity.py against one library (RAFTSIM_LIB)."""
import os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import numpy as np
import helpers
from test_gpu_parity import CASES
from raftsim._backend import Backend
lib, name = sys.argv[1], sys.argv[2]
cfg = CASES[name]
g = Backend(lib, "raft_sim_", **cfg)
r = helpers.oracle(**cfg)
helpers.oracle_threads(r, helpers.cpu_threads())
g.step(20000); r.step(20000)
bad = np.nonzero(g.digest() != r.digest())[0]
print(Path(lib).name, name, "clusters differing:", len(bad), "counters equal:", g.counters() == r.counters(), flush=True)
