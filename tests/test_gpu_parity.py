"""GPU parity: libraftsim.so (HIP, gfx950) against the C oracle, bit-exact per cluster.

Every cluster's canonical digest (SIM_SPEC §6: node records, queues, logs, arena cursors, trace
hashes, checker state) and every counter must match. On a mismatch the failing cluster is re-run
alone tick by tick on both sides and the first divergent tick is reported with both states.
"""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

FAULTS = dict(drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
# SIM_SPEC D14/D15: bursts of client traffic with quiet gaps longer than the election timeout,
# and clients that follow redirect-client (server.clj:62-63) to the leader
BURSTS = dict(client_period=16384, client_burst=2048, client_redirects=4)
C4_BURSTS = dict(log_cap=4096, client_ppm=500000, client_period=8192, client_burst=2048,
                 client_redirects=4)

CASES = {
    # C2 shape (no faults, no client traffic), smaller cluster count
    "c2_small": dict(n_clusters=4096, nodes=5, seed=42),
    # C3 shape: faults, partitions, client-set
    "c3_faults": dict(n_clusters=2048, nodes=5, seed=1, client_ppm=1000, log_cap=256, **FAULTS),
    # C4 shape: 7 and 9 nodes, client-heavy, long logs
    "c4_n7": dict(n_clusters=1024, nodes=7, seed=3, client_ppm=3000, log_cap=512,
                  commit_stream_cap=256),
    "c4_n9": dict(n_clusters=512, nodes=9, seed=5, client_ppm=2000, log_cap=1024, dup_ppm=20000,
                  dmax=8),
    # C5: bug variant (vote granted without the log check)
    "c5_variant": dict(n_clusters=1024, nodes=5, seed=9, client_ppm=1000, log_cap=256,
                       variant_flags=1, commit_stream_cap=7, **FAULTS),
    # overflow and tiny inboxes, heavy duplication
    "overflow": dict(n_clusters=512, nodes=9, seed=11, inbox_cap=2, dup_ppm=300000, dmax=3,
                     client_ppm=5000, log_cap=64),
    # arena pressure: arena == 2L, short logs, frequent client-sets
    "arena_tight": dict(n_clusters=512, nodes=5, seed=13, client_ppm=20000, log_cap=16,
                        arena_cap=32, dup_ppm=100000, dmax=10),
    # arena sizes that are not a multiple of the 8-slot chunks of the arena loops (tick_wave.hpp):
    # runs wrap inside a chunk, and chunks read past an arena's end into the next one
    "arena_odd": dict(n_clusters=512, nodes=5, seed=14, client_ppm=20000, log_cap=16,
                      arena_cap=37, hb=40, el_base=60, el_span=60, dup_ppm=100000, dmax=10,
                      commit_stream_cap=5),
    "spec_arena_odd": dict(n_clusters=512, nodes=5, seed=15, client_ppm=30000, log_cap=24,
                           arena_cap=51, hb=40, el_base=60, el_span=60, variant_flags=2, **FAULTS),
    # launch boundaries that split ticks oddly
    "tiny_launches": dict(n_clusters=300, nodes=5, seed=17, client_ppm=1000, ticks_per_launch=7,
                          **FAULTS),
    "n2": dict(n_clusters=700, nodes=2, seed=19, client_ppm=500, **FAULTS),
    "n3": dict(n_clusters=700, nodes=3, seed=21, client_ppm=500, **FAULTS),
    "n4": dict(n_clusters=700, nodes=4, seed=23, client_ppm=500, **FAULTS),
    "n6": dict(n_clusters=700, nodes=6, seed=25, client_ppm=500, **FAULTS),
    "n8": dict(n_clusters=700, nodes=8, seed=27, client_ppm=500, **FAULTS),
    # F3 trace rings on (they enter the digest): wrap-around, entry-ring overwrite, evictions
    "traced": dict(n_clusters=1024, nodes=5, seed=31, client_ppm=2000, log_cap=128, trace_cap=48,
                   trace_entry_cap=300, commit_stream_cap=16, **FAULTS),
    "traced_tight": dict(n_clusters=256, nodes=9, seed=33, client_ppm=20000, log_cap=16,
                         arena_cap=32, dup_ppm=100000, dmax=10, trace_cap=16, trace_entry_cap=64),
    "fast_timers": dict(n_clusters=1000, nodes=5, seed=29, hb=30, el_base=50, el_span=50,
                        client_ppm=20000, log_cap=128, **FAULTS),
    # F4 Spec-Raft control (SIM_SPEC §8) and its bug-injected form
    "spec_c3": dict(n_clusters=2048, nodes=5, seed=41, client_ppm=2000, log_cap=256,
                    variant_flags=2, commit_stream_cap=64, **FAULTS),
    "spec_nolog": dict(n_clusters=1024, nodes=5, seed=43, client_ppm=5000, log_cap=512, hb=300,
                       el_base=500, el_span=500, variant_flags=3, **FAULTS),
    "spec_n9": dict(n_clusters=512, nodes=9, seed=45, client_ppm=3000, log_cap=1024,
                    variant_flags=2, commit_stream_cap=256, dup_ppm=20000, dmax=8),
    "spec_n4_traced": dict(n_clusters=512, nodes=4, seed=47, client_ppm=4000, log_cap=128,
                           variant_flags=2, trace_cap=32, trace_entry_cap=256, **FAULTS),
    "spec_tight": dict(n_clusters=512, nodes=3, seed=49, client_ppm=30000, log_cap=24,
                       arena_cap=48, hb=40, el_base=60, el_span=60, variant_flags=2,
                       inbox_cap=3, **FAULTS),
    # BASELINE config 4: 7 and 9 nodes, 4096-entry logs, bursts that build 1000+-entry batches
    "c4_n7_bursts": dict(n_clusters=512, nodes=7, seed=3, commit_stream_cap=256, **C4_BURSTS),
    "c4_n9_bursts": dict(n_clusters=256, nodes=9, seed=5, dup_ppm=20000, dmax=8, **C4_BURSTS),
    # the N >= 7 burst engine's edges (tick_wave.hpp BURST): no redirect hops (abandoned
    # client-sets) with one-slot inboxes; follower timers and heartbeats that fall inside bursts;
    # launches that split bursts at odd ticks
    "burst_edges_n7": dict(n_clusters=512, nodes=7, seed=91, client_ppm=500000, client_period=4096,
                           client_burst=1024, client_redirects=0, inbox_cap=1, log_cap=700, hb=300,
                           el_base=500, el_span=500),
    "burst_timers_n9": dict(n_clusters=512, nodes=9, seed=93, client_ppm=300000, client_period=2048,
                            client_burst=512, client_redirects=1, inbox_cap=2, log_cap=2000, hb=40,
                            el_base=60, el_span=40),
    "burst_launches_n8": dict(n_clusters=512, nodes=8, seed=95, client_ppm=500000,
                              client_period=1024, client_burst=256, client_redirects=4,
                              ticks_per_launch=37, log_cap=1500),
    # config 3 / 5 shapes with the bursty, redirect-following client
    "c3_bursts": dict(n_clusters=2048, nodes=5, seed=1, client_ppm=80000, log_cap=256,
                      **BURSTS, **FAULTS),
    "spec_bursts": dict(n_clusters=1024, nodes=5, seed=61, client_ppm=80000, log_cap=1024,
                        variant_flags=2, commit_stream_cap=64, **BURSTS, **FAULTS),
    "spec_nolog_bursts": dict(n_clusters=1024, nodes=5, seed=63, client_ppm=80000, log_cap=1024,
                              variant_flags=3, **BURSTS, **FAULTS),
    # faithful crash storm under client traffic: most client-sets reach halted nodes (to-halted)
    "crash_storm_clients": dict(n_clusters=2048, nodes=5, seed=13, client_ppm=80000, log_cap=16,
                                hb=300, el_base=500, el_span=500, **BURSTS, **FAULTS),
    "redirect_storm": dict(n_clusters=512, nodes=6, seed=65, client_ppm=1000000,
                           client_period=300, client_burst=40, client_redirects=16, inbox_cap=4,
                           log_cap=128, hb=50, el_base=80, el_span=80, **FAULTS),
    # LITE launches (no faults, no client, fixed delay) at N <= 5 take the steady kernel and hand
    # every other event to the catch-up launch (steady_kernel.hip): its edges
    "lite_n2": dict(n_clusters=1000, nodes=2, seed=71, hb=40, el_base=60, el_span=40),
    "lite_n3": dict(n_clusters=1000, nodes=3, seed=73, hb=300, el_base=500, el_span=500),
    "lite_n4": dict(n_clusters=1000, nodes=4, seed=75, hb=300, el_base=500, el_span=500, dmin=4,
                    dmax=4),
    # heartbeats slower than the election timer: elections keep interrupting the rounds
    "lite_elections": dict(n_clusters=1200, nodes=5, seed=77, hb=700, el_base=500, el_span=400,
                           dmin=3, dmax=3),
    # two-slot inboxes: a leader's four responses overflow its RES ring (the slow delivery path)
    "lite_tiny_inbox": dict(n_clusters=1200, nodes=5, seed=79, inbox_cap=2, hb=200, el_base=500,
                            el_span=300),
    # odd launch splits: queued messages cross launch boundaries into the pair cells
    "lite_odd_launches": dict(n_clusters=600, nodes=5, seed=81, ticks_per_launch=13, hb=60,
                              el_base=100, el_span=100, dmin=7, dmax=7),
    # timers too short for the lane kernel's one-trip heartbeat round (hb < 2d + N - 1, el_base <
    # d + N - 1): every round runs tick by tick, elections keep interrupting them
    "lite_short_round": dict(n_clusters=1000, nodes=5, seed=85, hb=9, el_base=6, el_span=30,
                             dmin=3, dmax=3),
}


def run_pair(cfg, ticks, chunk):
    g = helpers.gpu(**cfg)
    r = helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    done = 0
    while done < ticks:
        n = min(chunk, ticks - done)
        g.step(n)
        r.step(n)
        done += n
        dg, dr = g.digest(), r.digest()
        bad = np.nonzero(dg != dr)[0]
        if len(bad):
            c = int(bad[0])
            msg = (f"{len(bad)} of {cfg['n_clusters']} clusters differ after {done} ticks; "
                   f"first local cluster {c}\n" + helpers.describe_cluster_diff(g, r, c) + "\n"
                   + helpers.bisect_divergence(cfg, cfg.get("cluster_offset", 0) + c, done,
                                               helpers.gpu, helpers.oracle))
            pytest.fail(msg)
    return g, r


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_matches_oracle(name):
    cfg = CASES[name]
    g, r = run_pair(cfg, 20000, 5000)
    cg, cr = g.counters(), r.counters()
    assert cg == cr
    assert cg["node_ticks"] == cfg["n_clusters"] * cfg["nodes"] * 20000


@pytest.mark.parametrize("seed", [1, 42, 0xDEADBEEF, 0x1_2345_6789])
def test_gpu_c2_full_size(seed):
    """BASELINE config 2: 65,536 five-node clusters, no faults, for the seeds of SURVEY §8(d) and
    one above 2^32 (Philox key word 1 nonzero): digest-equal after each of four 10k-tick launches.
    The first launch (elections) runs the steady kernel, which runs init-node's election in closed
    form, two timers firing together included (about 30 clusters per seed; only three together
    would be handed to the general body); the last one is the steady kernel alone on the
    256-workgroup grid with no cluster bailed (core.clj:91-139,105-123,141-149,162-169,181)."""
    cfg = dict(n_clusters=65536, nodes=5, seed=seed)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    bails = []
    for launch in range(4):
        g.step(10000)
        r.step(10000)
        bails.append(g.diag_last_bails())
        bad = np.nonzero(g.digest() != r.digest())[0]
        assert not len(bad), f"launch {launch}: {len(bad)} clusters differ, first {bad[0]}"
    assert g.counters() == r.counters()
    assert 0 <= bails[0] <= 2 and bails[-1] == 0, bails


@pytest.mark.parametrize("variant,nodes", [(0, 5), (2, 5), (3, 5), (0, 9), (2, 7)])
def test_gpu_storm_window(variant, nodes):
    """The STORM body (tick_wave.hpp): a fresh handle with client traffic runs the ticks before
    el_base -- where only client-sets at followers and their redirects can happen -- as a launch of
    its own, split off the first step; digest- and counter-equal to the oracle after it and after
    the elections that follow (core.clj:151-160 with server.clj:62-63; 166-169). A host write of the
    clock ends the storm ticks: the same step is then one launch, with the same results."""
    cfg = dict(n_clusters=4096, nodes=nodes, seed=11 + variant, hb=400, el_base=1500, el_span=800,
               client_ppm=300000, client_period=4096, client_burst=1024, client_redirects=4,
               log_cap=256, variant_flags=variant, drop_ppm=50000, dmin=1, dmax=20)
    r = helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    g = helpers.gpu(ticks_per_launch=4000, **cfg)
    g.step(4000)
    r.step(4000)
    assert g.last_step_timing()[1] == 2                  # [0, 1500) storm, then [1500, 4000)
    assert np.array_equal(g.digest(), r.digest())
    g.step(4000)
    r.step(4000)
    assert g.last_step_timing()[1] == 1
    assert np.array_equal(g.digest(), r.digest())
    c = g.counters()
    assert c == r.counters() and c["redirects"] > 0 and c["leaders"] > 0
    g.close()
    g2 = helpers.gpu(ticks_per_launch=4000, **cfg)
    g2.set_tick(0)                                       # a host write of the clock
    g2.step(4000)
    assert g2.last_step_timing()[1] == 1
    r2 = helpers.oracle(**cfg)
    helpers.oracle_threads(r2, helpers.cpu_threads())
    r2.step(4000)
    assert np.array_equal(g2.digest(), r2.digest())


@pytest.mark.parametrize("variant,inbox,nodes", [(0, 16, 5), (2, 2, 5), (0, 16, 3), (2, 16, 9),
                                                 (0, 3, 9)])
def test_gpu_storm_engine(variant, inbox, nodes):
    """The storm kernel (storm_kernel.hip, one lane per cluster; handles of 131,072 clusters or
    more, every N from 2 to 9): storm launches split into chunks (rings carried across launches),
    with small inboxes whose overflowing clusters are rerun by the lane-per-node STORM body;
    digest- and counter-equal to the oracle through the storm ticks and the elections after them
    (core.clj:151-160, server.clj:62-63). The storm kernel's leftover list stays a minority with
    the default inbox (a regression to rerunning most clusters would show here)."""
    cfg = dict(n_clusters=131072, nodes=nodes, seed=21 + variant + nodes, el_base=3000,
               el_span=2000, client_ppm=200000, client_period=8192, client_burst=2048,
               client_redirects=4, inbox_cap=inbox, log_cap=128, variant_flags=variant,
               drop_ppm=100000, dmin=1, dmax=30, part_ppm=50000)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    bails = []
    for _ in range(4):
        g.step(1250)
        r.step(1250)
        if g.tick <= 3000 + 1250:
            bails.append(g.diag_storm_bails())
        bad = np.nonzero(g.digest() != r.digest())[0]
        assert not len(bad), f"tick {g.tick}: {len(bad)} clusters differ, first {bad[0]}"
    assert g.counters() == r.counters()
    assert bails and min(bails) >= 0, bails              # the storm kernel ran every storm launch
    if inbox >= 16:
        assert max(bails) < 131072 // 4, bails


@pytest.mark.parametrize("nodes,d", [(2, 1), (3, 2), (4, 1), (5, 3), (5, 1)])
def test_gpu_init_election_closed_form(nodes, d):
    """The steady kernel's election from init-node (steady_kernel.hip) for every follower count
    and a delay above 1 (the electing vote response and the first append-response tick move with
    both): short timers so that elections, the first heartbeat rounds and the ties it hands to the
    general body all fall inside the first launch; digest- and counter-equal to the oracle after
    each launch, with few clusters bailed (core.clj:91-139,166-169)."""
    cfg = dict(n_clusters=16384, nodes=nodes, seed=7 + nodes, hb=300, el_base=700, el_span=900,
               dmin=d, dmax=d)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    bails = []
    for launch in range(3):
        g.step(3000)
        r.step(3000)
        bails.append(g.diag_last_bails())
        bad = np.nonzero(g.digest() != r.digest())[0]
        assert not len(bad), f"launch {launch}: {len(bad)} clusters differ, first {bad[0]}"
    assert g.counters() == r.counters()
    assert 0 <= bails[0] < 16384 // 20, bails


def _client_set_into(be, cluster, node, value):
    """Append a client-set (SIM_SPEC §3, server.clj:12) to a node's REQ queue, arriving now."""
    q = [list(m) for m in be.read_queue(cluster, node, 0)]
    arr = max([be.tick] + [m[0] for m in q])
    be.write_queue(cluster, node, 0, q + [[arr, 3, 0, value, 0, 0, 0, 0]])


@pytest.mark.parametrize("mode", ["auto", "always"])
@pytest.mark.parametrize("event", ["set_tick", "client_set", "client_cursor", "node_term",
                                   "node_log"])
def test_gpu_host_writes_after_lite_launches(event, mode, monkeypatch):
    """Host writes after 14 LITE launches (past the 8-launch packing period, with the packing
    reused between rebuilds): set_tick, a queued client-set and a finite client cursor (both clear
    LITE for the rest of the handle), and node records rewritten under clusters the steady kernel
    left with a certificate (a follower's term raised; a log entry given to a leader and committed:
    raft_sim_write_nodes clears the certificate, device.hpp) land at every phase of the rebuild
    cycle; GPU == oracle after each of the next 10 launches (raftsim.hip: packing keys and
    histogram stay consistent)."""
    monkeypatch.setenv("RAFTSIM_STEADY", mode)
    cfg = dict(n_clusters=4096, nodes=5, seed=42, ticks_per_launch=1000, log_cap=64)
    for phase in (0, 3):
        g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
        helpers.oracle_threads(r, helpers.cpu_threads())
        for _ in range(14 + phase):
            g.step(1000)
            r.step(1000)
        for be in (g, r):
            if event == "set_tick":
                be.set_tick(be.tick + 777)
            elif event == "client_set":
                for c in (5, 100, 4095):
                    _client_set_into(be, c, 1 + c % 5, 1000 + c)
            elif event == "client_cursor":
                be.write_clusters(7, [dict(hwm=(0, 0, 0), client_next=be.tick + 100,
                                           client_count=0)])
            else:
                for c in (3, 200, 4000):
                    raw = be.read_nodes_raw(c, 1)
                    lead = next(i for i in range(5) if raw[i].role == 2)
                    if event == "node_term":           # a follower one term ahead
                        raw[(lead + 1) % 5].current_term += 1
                    else:                              # the leader's log gets a committed entry
                        be.write_arena(c, lead + 1, [(raw[lead].current_term, 77)])
                        raw[lead].log_len = 1
                        raw[lead].commit_index = 1
                        raw[lead].arena_base = 0
                        raw[lead].arena_frontier = 1
                    be.write_nodes(c, raw)
        for launch in range(10):
            g.step(1000)
            r.step(1000)
            bad = np.nonzero(g.digest() != r.digest())[0]
            assert not len(bad), f"launch {launch}: {len(bad)} clusters differ, first {bad[0]}"
        assert g.counters() == r.counters()


@pytest.mark.parametrize("nodes", [7, 9])
def test_gpu_c4_logs_reach_capacity(nodes):
    """BASELINE config 4 to its end: 4096-entry logs fill up under the bursty client, append-entries
    carry 1000+ entries (core.clj:56-67 ships the whole suffix), and OVERFLOW halts appear (D8);
    GPU == oracle on every cluster, counter and the payload maximum."""
    cfg = dict(n_clusters=64, nodes=nodes, seed=7 + nodes, **C4_BURSTS)
    g, r = run_pair(cfg, 110000, 55000)
    cg, cr = g.counters(), r.counters()
    assert cg == cr
    assert cg["payload_max"] >= 1000 and cg["halt_overflow"] > 0
    assert max(n["log_len"] for n in g.read_nodes()) >= 3000


def test_gpu_sharded_handle_equals_single():
    """n_devices = 3 (three shards; on a one-GPU box they share the device) reproduces the
    one-shard handle: digests, counters, reads that cross shard boundaries, and resume."""
    cfg = dict(n_clusters=1000, nodes=5, seed=71, client_ppm=80000, log_cap=256, **BURSTS,
               **FAULTS)
    one, three = helpers.gpu(**cfg), helpers.gpu(n_devices=3, **cfg)
    for s in (one, three):
        s.step(20000)
    assert np.array_equal(one.digest(), three.digest())
    assert one.counters() == three.counters()
    assert one.read_nodes(300, 100) == three.read_nodes(300, 100)
    assert one.read_clusters(330, 10) == three.read_clusters(330, 10)
    for c in (332, 333, 334, 666, 667):
        for i in (1, 5):
            assert one.read_queue(c, i, 0) == three.read_queue(c, i, 0)
            assert one.log(c, i) == three.log(c, i)


def test_gpu_printed_trace_matches_oracle():
    """F3: the `; Node` / `; Message` dump (core.clj:182-186) of GPU-recorded events equals the
    oracle's, text for text, on a faulty client-driven run."""
    cfg = dict(n_clusters=8, nodes=5, seed=35, client_ppm=3000, log_cap=256, trace_cap=4096,
               trace_entry_cap=1 << 15, **FAULTS)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    g.step(20000)
    r.step(20000)
    n_entries = 0
    for c in range(cfg["n_clusters"]):
        for i in range(1, 6):
            tg = g.edn_trace(c, i)
            assert tg == r.edn_trace(c, i), (c, i)
            n_entries += tg.count(":val ")
    assert n_entries > 0


def test_gpu_spec_raft_safety_at_scale():
    """BASELINE config 5 shape on the GPU: 65,536 Spec-Raft clusters with faults, client traffic
    and fast timers show no violation (control), while the same clusters with the up-to-date vote
    check dropped do; both bit-exact against the oracle on a sampled slice."""
    base = dict(n_clusters=65536, nodes=5, seed=51, client_ppm=5000, log_cap=256, hb=300,
                el_base=500, el_span=500, **FAULTS)
    ctl, bug = helpers.gpu(variant_flags=2, **base), helpers.gpu(variant_flags=3, **base)
    for s in (ctl, bug):
        s.step(20000)
    c, b = ctl.counters(), bug.counters()
    assert c["leaders"] > 100000 and c["viol_election"] == c["viol_log"] == c["viol_complete"] == 0
    assert b["viol_complete"] > 0 and b["first_violation_tick"] is not None
    lo = 4096
    for flags, sim in ((2, ctl), (3, bug)):
        r = helpers.oracle(**dict(base, n_clusters=lo, variant_flags=flags))
        helpers.oracle_threads(r, helpers.cpu_threads())
        r.step(20000)
        assert np.array_equal(sim.digest(0, lo), r.digest())


def test_gpu_shard_invariance():
    """Two handles over disjoint cluster ranges reproduce one handle over both (D13)."""
    base = dict(nodes=5, seed=99, client_ppm=1000, log_cap=128, **FAULTS)
    whole = helpers.gpu(n_clusters=600, **base)
    lo = helpers.gpu(n_clusters=250, cluster_offset=0, **base)
    hi = helpers.gpu(n_clusters=350, cluster_offset=250, **base)
    for s in (whole, lo, hi):
        s.step(12000)
    assert np.array_equal(whole.digest(), np.concatenate([lo.digest(), hi.digest()]))
    cw, cl, ch = whole.counters(), lo.counters(), hi.counters()
    for k in cw:
        if k == "first_violation_tick":
            vals = [v for v in (cl[k], ch[k]) if v is not None]
            assert cw[k] == (min(vals) if vals else None)
        elif k == "payload_max":
            assert cw[k] == max(cl[k], ch[k])
        else:
            assert cw[k] == cl[k] + ch[k], k


def test_gpu_write_state_roundtrip():
    """State written through the ABI reads back identically and steps like the oracle."""
    cfg = dict(n_clusters=64, nodes=5, seed=3, client_ppm=3000, log_cap=64, **FAULTS)
    src = helpers.oracle(**cfg)
    src.step(15000)
    g = helpers.gpu(**cfg)
    r = helpers.oracle(**cfg)
    for be in (g, r):
        be.set_tick(15000)                       # resume: deadlines are absolute ticks
        be.write_nodes(0, src.read_nodes_raw())
        be.write_clusters(0, src.read_clusters())
        for c in range(cfg["n_clusters"]):
            for i in range(1, 6):
                be.write_arena(c, i, src.read_arena(c, i))
                for w in (0, 1):
                    be.write_queue(c, i, w, src.read_queue(c, i, w))
    assert np.array_equal(g.digest(), src.digest())
    for be in (g, r, src):
        be.step(8000)
    assert np.array_equal(g.digest(), r.digest())
    assert np.array_equal(g.digest(), src.digest())     # resumed == never stopped


def test_gpu_multi_launch_step():
    """One raft_sim_step spanning several launches (ticks_per_launch < n_ticks) equals the oracle."""
    cfg = dict(n_clusters=512, nodes=5, seed=81, client_ppm=20000, log_cap=64,
               ticks_per_launch=3000, **BURSTS, **FAULTS)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    g.step(17000)
    r.step(17000)
    assert g.tick == r.tick == 17000
    assert np.array_equal(g.digest(), r.digest()) and g.counters() == r.counters()


def test_gpu_tick_horizon():
    """No deadline or arrival may wrap past 2^32 (SIM_SPEC D1): steps that could are refused."""
    g = helpers.gpu(n_clusters=64, nodes=5, seed=1)
    top = 2 ** 32 - 1 - 10000        # the longest timer is el_base + el_span = 10000
    g.set_tick(top - 3000)
    g.step(2999)
    with pytest.raises(helpers.RaftSimError, match="2\\^32"):
        g.step(2)
    g.step(0)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    dict(n_clusters=4096, nodes=5, seed=42),
    dict(n_clusters=2048, nodes=7, seed=3, client_ppm=20000, log_cap=128, **FAULTS),
    dict(n_clusters=1024, nodes=5, seed=41, client_ppm=2000, log_cap=256, variant_flags=2,
         commit_stream_cap=64, **FAULTS),
], ids=["c2_shape", "faults_n7", "spec"])
def test_gpu_schedule_invariance(cfg):
    """RAFT_SCHED_ALIGNED (clusters regrouped onto waves by next event before every launch) and
    RAFT_SCHED_FIXED produce the same per-cluster digests and counters, launch by launch."""
    a = helpers.gpu(**cfg, schedule=0, ticks_per_launch=2500)
    b = helpers.gpu(**cfg, schedule=1, ticks_per_launch=2500)
    for _ in range(4):
        a.step(5000)
        b.step(5000)
        assert np.array_equal(a.digest(), b.digest())
        assert a.counters() == b.counters()


@pytest.mark.gpu
def test_gpu_step_async_matches_step():
    """K raft_sim_step_async calls + one raft_sim_sync leave the same state, counters and tick as
    K synchronous raft_sim_step calls, and the timing covers every launch of the K steps."""
    cfg = dict(n_clusters=2048, nodes=5, seed=9, client_ppm=5000, log_cap=128,
               ticks_per_launch=3000, **FAULTS)
    a, b = helpers.gpu(**cfg), helpers.gpu(**cfg)
    for _ in range(4):
        a.step(5000)
        b.step_async(5000)
    b.sync()
    assert a.tick == b.tick == 20000
    assert np.array_equal(a.digest(), b.digest())
    assert a.counters() == b.counters()
    ms, launches = b.last_step_timing()
    assert launches == 8 and ms > 0


@pytest.mark.parametrize("ppm", [0, 30000])
def test_gpu_host_written_client_cursor(ppm):
    """A client cursor written by the host (checkpoint/resume through raft_sim_write_clusters) is
    honoured like any other, also with client_ppm = 0, where every power of the gap search is
    2^32 and the next injection never comes (SIM_SPEC §4 P0)."""
    cfg = dict(n_clusters=64, nodes=5, seed=77, client_ppm=ppm, log_cap=64)
    g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
    recs = [dict(hwm=(0, 0, 0), client_next=100 + 37 * i, client_count=i) for i in range(64)]
    g.write_clusters(0, recs)
    r.write_clusters(0, recs)
    for _ in range(3):
        g.step(4000)
        r.step(4000)
        assert (g.digest() == r.digest()).all()
    assert g.counters() == r.counters()
    assert g.counters()["client_injected"] >= 64




def test_gpu_steady_path_taken():
    """C2 from init-node: the first launch takes the steady path with the elections in closed form
    (at most a couple of tied clusters bailed to the general body); once every cluster has its
    leader the steady kernel runs every cluster alone (0 bails); the state equals the oracle's
    after every launch."""
    cfg = dict(n_clusters=8192, nodes=5, seed=83)
    g = helpers.gpu(**cfg)
    r = helpers.oracle(**cfg)
    helpers.oracle_threads(r, helpers.cpu_threads())
    bails = []
    for _ in range(4):
        g.step(10000)
        r.step(10000)
        bails.append(g.diag_last_bails())
        assert (g.digest() == r.digest()).all()
    assert g.counters() == r.counters()
    assert 0 <= bails[0] <= 2 and bails[-1] == 0, bails


LITE_CASES = ["c2_small", "lite_n2", "lite_n3", "lite_n4", "lite_elections", "lite_tiny_inbox",
              "lite_odd_launches", "lite_short_round"]


@pytest.mark.parametrize("name", LITE_CASES)
def test_gpu_forced_steady_matches_oracle(name, monkeypatch):
    """Every LITE launch on the steady kernel (RAFTSIM_STEADY=always), from init-node: elections
    and every other event outside its model go through the workgroup's catch-up (the general
    tick body over the clusters it bailed, several wave slots per wave); GPU == oracle after
    every chunk."""
    monkeypatch.setenv("RAFTSIM_STEADY", "always")
    cfg = CASES[name]
    g, r = run_pair(cfg, 20000, 5000)
    assert g.counters() == r.counters()
    assert g.diag_last_bails() >= 0          # the last launch took the steady path
