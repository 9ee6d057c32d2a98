"""The N>1 path on the GPU: two ranks (one process each, both on the box's one MI355X, gloo for the
host-side reduction -- RCCL needs one GPU per rank) each run their contiguous cluster shard through
libraftsim.so and all-reduce the counters exactly as bench.py does; digests and reduced counters
must equal one handle simulating every cluster (Philox is keyed by the global cluster id)."""
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

import helpers

pytestmark = pytest.mark.gpu

CFG = dict(nodes=5, seed=17, client_ppm=80000, client_period=16384, client_burst=2048,
           client_redirects=4, drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50,
           part_ppm=100000, log_cap=256)
TOTAL, STEPS = 20000, 3


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "raft-simulation_amd"), str(root / "tests"), str(root / "oracle")]
    import torch.distributed as dist
    import raftsim
    from raftsim import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = rdist.shard(TOTAL, rank, world)
    sim = raftsim.Simulator(n_clusters=cnt, cluster_offset=off, **CFG)
    for _ in range(STEPS):
        sim.step(10000)
    np.save(Path(out) / f"digest_{rank}.npy", sim.digest())
    red = rdist.reduce_counters(sim.counters())
    if rank == 0:
        (Path(out) / "counters.json").write_text(json.dumps(red))
    sim.close()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_two_ranks_equal_one_handle(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    whole = helpers.gpu(n_clusters=TOTAL, **CFG)
    for _ in range(STEPS):
        whole.step(10000)
    dg = np.concatenate([np.load(tmp_path / f"digest_{r}.npy") for r in range(2)])
    assert np.array_equal(dg, whole.digest())
    got = json.loads((tmp_path / "counters.json").read_text())
    assert got == whole.counters() and got["client_injected"] > 0
