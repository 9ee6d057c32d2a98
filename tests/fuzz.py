"""Random valid cluster states for differential testing (test infrastructure).

A batch shares one configuration; each cluster gets an independent random state that exercises
handler edge cases: every role incl. `:follwer`, terms in a narrow band, logs over a tiny entry
alphabet (so entry equalities and prev-log mismatches are frequent), commit beyond the log,
LazySeq logs, partial leader-states, negative next-index, halted nodes, and queued messages of all
five types with random arrivals (AppendEntries payloads are suffixes of the sender's log).
"""
from __future__ import annotations

import random

import scenarios
from scenarios import Scenario, msg, node

TYPES_REQ = ("request-vote", "append-entries", "client-set")
TYPES_RES = ("vote-response", "append-response")


def random_config(rng):
    n = rng.randint(2, 9)
    cfg = dict(nodes=n, seed=rng.getrandbits(64), log_cap=rng.choice([6, 8, 12]),
               inbox_cap=rng.randint(4, 16), hb=rng.randint(1, 6), el_base=rng.randint(1, 6),
               el_span=rng.randint(1, 6), variant_flags=rng.choice([0, 0, 0, 1, 2, 3]),
               commit_stream_cap=rng.choice([0, 2, 16]), trace_cap=rng.choice([0, 2, 64]))
    cfg["trace_entry_cap"] = rng.choice([0, 1, 4096]) if cfg["trace_cap"] else 0
    if rng.random() < 0.5:
        cfg.update(drop_ppm=rng.choice([0, 100000, 400000]), dup_ppm=rng.choice([0, 300000]),
                   dmin=1, dmax=rng.randint(1, 4))
    if rng.random() < 0.3:
        cfg.update(part_ppm=500000, part_epoch=rng.randint(1, 4))
    if rng.random() < 0.3:
        cfg["client_ppm"] = rng.choice([100000, 500000])
    cfg["client_redirects"] = rng.choice([0, 0, 1, 3])
    if rng.random() < 0.2:
        cfg.update(client_period=rng.randint(2, 9), client_burst=1)
    return cfg


def _entry(rng):
    return (rng.randint(1, 3), rng.randint(0, 2))


def random_state(rng, cfg):
    N, L = cfg["nodes"], cfg["log_cap"]
    roles = ["follower", "candidate", "leader", "follwer"]
    nodes = {}
    for i in range(1, N + 1):
        peers = [p for p in range(1, N + 1) if p != i]
        role = rng.choice(roles)
        log = [_entry(rng) for _ in range(rng.randint(0, min(L, 5)))]
        if role == "leader":
            ls = {p: (rng.randint(-2, len(log) + 2), rng.randint(0, 4)) for p in peers}
        elif rng.random() < 0.3:
            ls = {p: (rng.randint(-1, 4), rng.randint(0, 4)) for p in rng.sample(peers, rng.randint(0, len(peers)))}
        else:
            ls = None
        nodes[i] = node(role, term=rng.randint(1, 4), voted_for=rng.randint(0, N),
                        leader_id=rng.randint(0, N),
                        votes=rng.sample(range(1, N + 1), rng.randint(0, N)), ls=ls, log=log,
                        commit=rng.randint(0, len(log) + 1), is_seq=int(rng.random() < 0.2),
                        deadline=rng.randint(0, 6), fault=int(rng.random() < 0.05),
                        last_led=rng.randint(0, 3))
    queues = {}
    for i in range(1, N + 1):
        for which, types in ((0, TYPES_REQ), (1, TYPES_RES)):
            cnt = rng.randint(0, min(3, cfg["inbox_cap"]))
            arrivals = sorted(rng.randint(0, 4) for _ in range(cnt))
            ms = [_random_msg(rng, rng.choice(types), a, i, N, nodes) for a in arrivals]
            if ms:
                queues[(i, which)] = ms
    hwm = (0, 0, 0)
    if rng.random() < 0.5:
        hwm = (rng.randint(1, 3), rng.randint(1, 3), rng.randint(0, 2))
    return nodes, queues, hwm


def _random_msg(rng, typ, arrival, dst, N, nodes):
    src = rng.choice([p for p in range(1, N + 1) if p != dst])
    term = rng.randint(1, 5)
    if typ == "client-set":
        return msg(typ, arrival, command=rng.randint(0, 2), hops=rng.randint(0, 3))
    if typ == "request-vote":
        return msg(typ, arrival, term=term, candidate_id=src, last_log_index=rng.randint(0, 4),
                   last_log_term=None if rng.random() < 0.3 else _entry(rng))
    if typ == "append-entries":
        slog = nodes[src]["log"]
        k = rng.randint(0, len(slog))
        return msg(typ, arrival, term=term, leader_id=src, leader_commit=rng.randint(0, 4),
                   prev_log_index=rng.randint(0, 4),
                   prev_log_term=None if rng.random() < 0.3 else _entry(rng),
                   entries=slog[len(slog) - k:])
    if typ == "vote-response":
        return msg(typ, arrival, term=term, id=src, vote_granted=rng.random() < 0.6)
    if rng.random() < 0.6:
        return msg(typ, arrival, term=term, id=src, success=True, commit=rng.randint(0, 4),
                   log_index=rng.randint(0, 5))
    return msg(typ, arrival, term=term, id=src, success=False)


def random_scenario(rng, cfg=None):
    cfg = cfg or random_config(rng)
    nodes, queues, hwm = random_state(rng, cfg)
    extra = {k: v for k, v in cfg.items() if k != "nodes"}
    return Scenario(cfg["nodes"], nodes, queues, hwm, **extra)


def load_batch(make, cfg, scns):
    """One backend with len(scns) clusters, cluster c holding scenario c's state."""
    be = make(**dict(scns[0].cfg, n_clusters=len(scns)))
    for c, scn in enumerate(scns):
        scn.load_into(be, c)
    return be


__all__ = ["random_config", "random_scenario", "load_batch", "scenarios"]
