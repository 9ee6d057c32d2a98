"""Runs a fuzz batch against a sanitizer build of the oracle (ASan+UBSan or TSan).

Started by tests/test_sanitizers.py in a child process with the sanitizer runtime preloaded:
    LD_PRELOAD=<libasan.so|libtsan.so> python tests/sanitize_driver.py LIB SEED
Random configurations (every variant, client model, fault and ring setting) and random states
(tests/fuzz.py) are stepped with several threads, then every read path of the ABI is exercised.
"""
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]

import fuzz  # noqa: E402
import test_oracle  # noqa: E402
from raftsim._backend import Backend  # noqa: E402

lib, seed = sys.argv[1], int(sys.argv[2])
rng = random.Random(seed)


def make(**cfg):
    return Backend(lib, "raft_ref_", **cfg)


def exercise(be, clusters):
    be.step(1500)
    be.digest()
    be.counters()
    be.read_nodes()
    be.read_clusters()
    for c in range(min(clusters, 4)):
        for i in range(1, be.N + 1):
            be.read_queue(c, i, 0)
            be.read_queue(c, i, 1)
            be.log(c, i)
            be.commit_stream(c, i)
            if be.config.trace_cap:
                be.edn_trace(c, i)


for k in range(6):                      # random configurations from init-node
    cfg = test_oracle.random_config(rng)
    be = make(n_clusters=23, n_devices=rng.choice([1, 3]), **cfg)
    be._lib.raft_ref_set_threads(be._h, 4)
    be._lib.raft_ref_set_idle_skip(be._h, k % 2)
    exercise(be, 23)
for k in range(4):                      # random states (every role, LazySeq, partial leader-state)
    cfg = fuzz.random_config(rng)
    scns = [fuzz.random_scenario(rng, cfg) for _ in range(16)]
    be = fuzz.load_batch(make, cfg, scns)
    be._lib.raft_ref_set_threads(be._h, 4)
    exercise(be, 16)
print("sanitize driver ok", flush=True)
