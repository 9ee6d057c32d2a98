"""The N>1 path on CPU: gloo, world_size 2. Each rank simulates its cluster shard (oracle backend)
and the counters are all-reduced exactly as bench.py does over RCCL; the result must equal one
process simulating every cluster."""
import json
import os
import socket
import sys
from pathlib import Path

import torch.multiprocessing as mp

import helpers

CFG = dict(nodes=5, seed=11, client_ppm=1000, drop_ppm=50000, dup_ppm=10000, dmax=20,
           part_ppm=100000, log_cap=64)
TOTAL, TICKS = 301, 12000


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "raft-simulation_amd"), str(root / "tests"), str(root / "oracle")]
    import torch.distributed as dist
    import helpers as h
    from raftsim import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = rdist.shard(TOTAL, rank, world)
    be = h.oracle(n_clusters=cnt, cluster_offset=off, **CFG)
    be.step(TICKS)
    red = rdist.reduce_counters(be.counters())
    slowest = rdist.reduce_max(1.0 + rank)
    if rank == 0:
        Path(out).write_text(json.dumps({"counters": red, "max": slowest}))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_counters_equal_single_process(tmp_path):
    out = tmp_path / "r.json"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    got = json.loads(out.read_text())
    whole = helpers.oracle(n_clusters=TOTAL, **CFG)
    whole.step(TICKS)
    assert got["counters"] == whole.counters()
    assert got["max"] == 2.0


def test_shard_ranges_cover_exactly():
    from raftsim import dist as rdist
    for total in (1, 7, 65536, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [rdist.shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _search_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "raft-simulation_amd"), str(root / "tests"), str(root / "oracle")]
    import torch.distributed as dist
    import helpers as h
    from raftsim import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = rdist.shard(VTOTAL, rank, world)
    be = h.oracle(n_clusters=cnt, cluster_offset=off, **VCFG)
    fv, ticks, _ = rdist.first_violation_search(be, 500, 40000, lambda x: rdist.reduce_min(x))
    if rank == 0:
        Path(out).write_text(json.dumps({"fv": fv, "ticks": ticks}))
    dist.destroy_process_group()


# BASELINE config 5 shape (Spec-Raft with the up-to-date vote check dropped) on few clusters
VCFG = dict(nodes=5, seed=43, client_ppm=5000, log_cap=512, hb=300, el_base=500, el_span=500,
            variant_flags=3, drop_ppm=100000, dup_ppm=10000, dmax=50, part_ppm=100000)
VTOTAL = 64


def test_violation_search_stops_every_rank_at_the_same_chunk(tmp_path):
    """bench.py's config-5 loop: ranks step their shards chunk by chunk and MIN-all-reduce the
    first-violation tick; the job stops in the chunk where any rank first counted one, and the
    tick equals one process's search over every cluster."""
    from raftsim import dist as rdist
    out = tmp_path / "v.json"
    mp.spawn(_search_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    got = json.loads(out.read_text())
    whole = helpers.oracle(n_clusters=VTOTAL, **VCFG)
    fv, ticks, _ = rdist.first_violation_search(whole, 500, 40000)
    assert fv is not None and got == {"fv": fv, "ticks": ticks}
