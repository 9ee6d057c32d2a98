"""Multi-GPU plumbing: cluster-range sharding and the counter all-reduce.

Clusters are independent and Philox streams are keyed by the global cluster id (SIM_SPEC D13),
so a rank simulates a contiguous range of clusters with no data-path exchange. The only
collective is the end-of-run reduction of the counter vector (SUM) and the first-violation tick
(MIN) and the largest append-entries payload (MAX): a few hundred bytes, latency-bound, over RCCL (torch.distributed backend "nccl") on the GPU
box or gloo in the CPU tests.
"""
from __future__ import annotations

NONE_TICK = 2 ** 63 - 1


def shard(total_clusters: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [offset, offset + count) range of global cluster ids owned by `rank`."""
    lo = total_clusters * rank // world
    hi = total_clusters * (rank + 1) // world
    return lo, hi - lo


def reduce_counters(c: dict, device=None) -> dict:
    """All-reduce a counters dict (raftsim Backend.counters()) over the default process group."""
    import torch
    import torch.distributed as dist

    names = sorted(k for k in c if k not in ("first_violation_tick", "payload_max"))
    v = torch.tensor([int(c[k]) for k in names], dtype=torch.int64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    pm = None
    if "payload_max" in c:
        pm = torch.tensor([int(c["payload_max"])], dtype=torch.int64, device=device)
        dist.all_reduce(pm, op=dist.ReduceOp.MAX)
    fv = c.get("first_violation_tick")
    f = torch.tensor([NONE_TICK if fv is None else int(fv)], dtype=torch.int64, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    out = dict(zip(names, (int(x) for x in v.tolist())))
    fmin = int(f.item())
    out["first_violation_tick"] = None if fmin == NONE_TICK else fmin
    if pm is not None:
        out["payload_max"] = int(pm.item())
    return out


def reduce_max(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def reduce_min(x: int, device=None) -> int:
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def first_violation_search(sim, chunk: int, max_ticks: int, reduce_min_fn=None):
    """Step `sim` (any raftsim Backend) `chunk` ticks at a time until a safety violation has been
    counted anywhere in the job (BASELINE config 5: time to the first violation). With
    `reduce_min_fn` (a MIN all-reduce over the ranks, e.g. `lambda x: reduce_min(x, dev)`) every
    rank stops after the same chunk: the one in which any rank first counted a violation.
    Returns (job's first violation tick or None, ticks stepped, timing) with timing = (device ms
    of the steps, summed tick-kernel ms, tick-kernel launches) on a GPU backend, zeros otherwise."""
    done, span, kms, launches = 0, 0.0, 0.0, 0
    timed = "last_span" in getattr(sim, "_fns", {})
    fv = NONE_TICK
    while done < max_ticks and fv == NONE_TICK:
        n = min(chunk, max_ticks - done)
        sim.step(n)
        done += n
        if timed:
            span += sim.last_span()
            ms, nl = sim.last_step_timing()
            kms += ms * nl
            launches += nl
        fv = sim.counters()["first_violation_tick"]
        fv = NONE_TICK if fv is None else int(fv)
        if reduce_min_fn is not None:
            fv = reduce_min_fn(fv)
    return (None if fv == NONE_TICK else fv), done, (span, kms, launches)
