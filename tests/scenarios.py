"""Known-answer scenarios derived by hand from the reference source.

Each scenario builds one cluster's exact state (node maps, logs, queued messages, timers), runs a
few ticks and checks the outcome the reference's code implies; every expectation cites the lines
it follows. A scenario can be loaded into the Python restatement (oracle/pyref.py) or into any
library implementing include/raftsim.h (the C oracle, or libraftsim.so on the GPU), so the same
hand-derived answers pin all three implementations.
"""
from __future__ import annotations

import pyref

BIG = 10 ** 8     # a deadline that never fires inside a scenario
ROLE = {"follower": 0, "candidate": 1, "leader": 2, "follwer": 3}


def node(role="follower", term=1, voted_for=0, leader_id=0, votes=(), ls=None, log=(),
         commit=0, is_seq=0, deadline=BIG, fault=0, last_led=0):
    """ls: None (nil leader-state) or {peer: (next, match)}."""
    return dict(role=ROLE[role], term=term, voted_for=voted_for, leader_id=leader_id,
                votes=tuple(votes), ls=ls, log=list(log), commit=commit, is_seq=is_seq,
                deadline=deadline, fault=fault, last_led=last_led)


def msg(type, arrival, **f):
    return dict(type=type, arrival=arrival, **f)


class Scenario:
    def __init__(self, N, nodes, queues=None, hwm=(0, 0, 0), **cfg):
        self.N, self.nodes, self.hwm = N, nodes, hwm
        self.queues = queues or {}
        self.cfg = dict(dict(nodes=N, n_clusters=1, log_cap=64, commit_stream_cap=64,
                             trace_cap=64, trace_entry_cap=256), **cfg)

    # ---------------------------------------------------------------- C ABI backends
    def load_backend(self, make):
        be = make(**self.cfg)
        self.load_into(be, 0)
        return be

    def load_into(self, be, c):
        """Write this scenario's state into cluster c of an existing backend."""
        recs = be.read_nodes_raw(c, 1)
        for i in range(1, self.N + 1):
            d, r = self.nodes[i], recs[i - 1]
            r.role, r.current_term = d["role"], d["term"]
            r.voted_for, r.leader_id = d["voted_for"], d["leader_id"]
            r.votes = sum(1 << v for v in d["votes"])
            r.fault, r.entries_is_seq = d["fault"], d["is_seq"]
            r.commit_index, r.log_len, r.deadline = d["commit"], len(d["log"]), d["deadline"]
            r.arena_base, r.arena_frontier = 0, len(d["log"])
            r.last_led_term = d["last_led"]
            r.ls_present, r.ls_keys = int(d["ls"] is not None), 0
            for p in range(self.N):
                r.next_index[p] = r.match_index[p] = 0
            for p, (nx, mt) in (d["ls"] or {}).items():
                r.ls_keys |= 1 << p
                r.next_index[p - 1], r.match_index[p - 1] = nx, mt
        be.write_nodes(c, list(recs))
        for i in range(1, self.N + 1):
            be.write_arena(c, i, self.nodes[i]["log"])
        for (i, which), msgs in self.queues.items():
            be.write_queue(c, i, which, [self._encode(m) for m in msgs])
        rec = be.read_clusters(c, 1)[0]
        rec["hwm"] = tuple(self.hwm)
        be.write_clusters(c, [rec])

    def _encode(self, m):
        pm = self._py_msg(m)
        arrival, hdr, term, a, b, et, ev, payload = pyref.encode_msg(m["arrival"], pm)
        poff = 0
        if payload:
            slog = self.nodes[pyref.msg_src(pm)]["log"]
            assert [tuple(e) for e in slog[len(slog) - len(payload):]] == payload, \
                "injected payloads must be a suffix of the sender's log"
            poff = len(slog) - len(payload)
        return (arrival, hdr, term, a, b, et, ev, poff)

    # ---------------------------------------------------------------- Python restatement
    @staticmethod
    def _py_msg(m):
        pm = {k.replace("_", "-"): v for k, v in m.items() if k != "arrival"}
        for key in ("last-log-term", "prev-log-term"):
            if key in pm and pm[key] is not None:
                pm[key] = tuple(pm[key])
        if "entries" in pm:
            pm["entries"] = [tuple(e) for e in pm["entries"]]
        return pm

    def load_py(self):
        cfg = pyref.default_config(**{k: v for k, v in self.cfg.items()
                                      if k in pyref.default_config()})
        pc = pyref.PyCluster(cfg, 0)
        names = {v: k for k, v in pyref.ROLE_CODE.items()}
        for i in range(1, self.N + 1):
            d = self.nodes[i]
            ls = None
            if d["ls"] is not None:
                ls = {"next-index": {p: nx for p, (nx, _) in d["ls"].items()},
                      "match-index": {p: mt for p, (_, mt) in d["ls"].items()}}
            pc.nodes[i] = {"id": i, "state": names[d["role"]], "current-term": d["term"],
                           "voted-for": d["voted_for"] or None,
                           "leader-id": d["leader_id"] or None, "leader-state": ls,
                           "votes": set(d["votes"])}
            lg = pc.logs[i]
            lg.entries, lg.is_seq, lg.commit_index = [tuple(e) for e in d["log"]], \
                bool(d["is_seq"]), d["commit"]
            pc.deadline[i], pc.fault[i], pc.last_led[i] = d["deadline"], d["fault"], d["last_led"]
        for (i, which), msgs in self.queues.items():
            q = pc.req[i] if which == 0 else pc.res[i]
            q[:] = [(m["arrival"], self._py_msg(m)) for m in msgs]
        pc.hwm = tuple(self.hwm)
        return pc


class PyView:
    """Uniform read access to a PyCluster, shaped like the Backend records."""

    def __init__(self, pc):
        self.pc = pc
        self.t = 0

    def step(self, n):
        for _ in range(n):
            self.pc.step(self.t)
            self.t += 1

    def node(self, i):
        return self.pc.canonical_node(i)

    def log(self, i):
        return [tuple(e) for e in self.pc.logs[i].entries]

    def counters(self):
        return dict(self.pc.cnt)

    def commit_stream(self, i):
        return list(self.pc.stream[i])

    def edn(self, i):
        return pyref.stdout_of(self.pc, i)


class BackendView:
    def __init__(self, be):
        self.be = be

    def step(self, n):
        self.be.step(n)

    def node(self, i):
        return self.be.read_nodes(0, 1)[i - 1]

    def log(self, i):
        return self.be.log(0, i)

    def counters(self):
        return self.be.counters()

    def commit_stream(self, i):
        return self.be.commit_stream(0, i)

    def edn(self, i):
        return self.be.edn_trace(0, i)


def run(scn, which, make=None):
    return PyView(scn.load_py()) if which == "py" else BackendView(scn.load_backend(make))


# ================================================================ the scenarios
E1, E2, E3 = (2, 10), (2, 20), (2, 30)


def kat_majority(view_of):
    """majority? (core.clj:19-21): |votes| >= ceil(N/2); N=4 needs only 2 (non-strict)."""
    assert [pyref.majority(range(n - 1), set(range(k))) for n, k in
            ((5, 3), (5, 2), (7, 4), (7, 3), (9, 5), (9, 4), (4, 2), (4, 1))] == \
        [True, False, True, False, True, False, True, False]
    for n, need in ((4, 2), (5, 3), (7, 4), (9, 5)):
        # candidate 1 holding need-2 grants besides itself; one more grant -> leader (core.clj:133-138)
        votes = [1] + list(range(2, need))
        nodes = {i: node() for i in range(1, n + 1)}
        nodes[1] = node("candidate", term=2, voted_for=1, votes=votes)
        q = {(1, 1): [msg("vote-response", 0, term=1, id=need, vote_granted=True)]}
        v = view_of(Scenario(n, nodes, q))
        v.step(1)
        r = v.node(1)
        assert r["role"] == ROLE["leader"] and r["votes"] == 0 and r["leader_id"] == 1, (n, r)
        # leader-state (core.clj:40-42): next = commit + 1 = 1, match 0 for every peer
        assert r["next_index"] == [0] + [1] * (n - 1) and r["match_index"] == [0] * n
        # one fewer grant stays candidate with the vote recorded (core.clj:134)
        nodes[1] = node("candidate", term=2, voted_for=1, votes=votes[:-1])
        v = view_of(Scenario(n, nodes, q))
        v.step(1)
        r = v.node(1)
        if need > 2:
            assert r["role"] == ROLE["candidate"] and r["votes"] == sum(1 << x for x in votes[:-1] + [need])


def kat_first_election(view_of):
    """Ideal network, 5 nodes from init-node (core.clj:31-38); node 3 times out first."""
    nodes = {i: node(deadline=BIG) for i in range(1, 6)}
    nodes[3] = node(deadline=0)
    v = view_of(Scenario(5, nodes))
    v.step(1)                                    # t0: timeout-handler (core.clj:166-169)
    a = v.node(3)
    assert (a["role"], a["current_term"], a["voted_for"], a["votes"]) == \
        (ROLE["candidate"], 2, 3, 1 << 3)        # follower->candidate (core.clj:69-73)
    v.step(1)                                    # t1: every voter runs request-vote-handler
    for i in (1, 2, 4, 5):
        r = v.node(i)
        # grant sets :voted-for but keeps the term (core.clj:97-103 never touches the term)
        assert (r["role"], r["current_term"], r["voted_for"]) == (ROLE["follower"], 1, 3), r
    v.step(1)                                    # t2: first grant (from id 1: sender order)
    assert v.node(3)["votes"] == (1 << 3) | (1 << 1)
    v.step(1)                                    # t3: second grant -> majority -> leader
    a = v.node(3)
    assert (a["role"], a["votes"], a["voted_for"], a["leader_id"]) == (ROLE["leader"], 0, 0, 3)
    assert a["next_index"] == [1, 1, 0, 1, 1] and a["match_index"] == [0] * 5
    v.step(1)                                    # t4: followers take the AppendEntries
    for i in (1, 2, 4, 5):
        r = v.node(i)
        # candidate->follower (:follwer, core.clj:76), term and leader from the message (122-123)
        assert (r["role"], r["current_term"], r["voted_for"], r["leader_id"]) == \
            (ROLE["follwer"], 2, 0, 3), r
    v.step(5)                                    # t5: 4th vote (no-op), t6..t9: four replies
    a = v.node(3)
    # next-index := log-index = prev 0 + 0 entries; match-index := commit 0 (core.clj:147-149)
    assert a["next_index"] == [0, 0, 0, 0, 0] and a["role"] == ROLE["leader"]
    c = v.counters()
    assert c["leaders"] == 1 and c["ev_vr"] == 4 and c["ev_ar"] == 4 and c["ev_ae"] == 4


def kat_duplication(view_of):
    """AppendEntries appends without truncation (log.clj:61-64) and ships prev+1 (core.clj:61,66)."""
    ls = {2: (1, 0), 3: (1, 0)}
    nodes = {1: node("leader", term=2, leader_id=1, ls=ls, log=[E1, E2, E3], deadline=0,
                     last_led=2),
             2: node("follwer", term=2, leader_id=1),
             3: node("follwer", term=2, leader_id=1)}
    v = view_of(Scenario(3, nodes))
    v.step(3)        # t0 heartbeat, t1 followers append, t2 leader takes reply from 2
    assert v.log(2) == [E2, E3] and v.node(2)["commit_index"] == 2    # e1 lost
    v.step(1)        # t3 reply from 3
    assert v.node(1)["next_index"][1:] == [2, 2]
    # second heartbeat 3000 ticks after the leader's last event (hb, core.clj:173): tick 3003,
    # delivered at 3004
    v.step(3001)
    assert v.log(2) == [E2, E3, E3] and v.log(3) == [E2, E3, E3]
    v.step(3003)
    assert v.log(2) == [E2, E3, E3, E3]         # one more e3 per heartbeat
    # node_2.log (log.clj:16-18,69-76): each apply writes the take-last `amount` :val's
    assert v.commit_stream(2) == [20, 30, 30, 30]
    assert v.counters()["viol_log"] >= 1        # same index and term, different value


def kat_truncate_crash(view_of):
    """Inconsistent AE: drop-last prev (log.clj:78-81), LazySeq; next timeout IOOBE (log.clj:47-49)."""
    X, Y, Z = (1, 7), (1, 8), (1, 9)
    # the sender has since crashed (halted), so no later heartbeat re-arms node 2's timer
    nodes = {1: node("leader", term=2, leader_id=1, ls={2: (3, 0)}, fault=1),
             2: node("follwer", term=2, leader_id=1, log=[X, Y, Z], commit=3)}
    q = {(2, 0): [msg("append-entries", 0, term=2, leader_id=1, leader_commit=0,
                      prev_log_index=2, prev_log_term=(5, 5), entries=[])]}
    nodes[2]["deadline"] = 1
    v = view_of(Scenario(2, nodes, q))
    v.step(1)
    r = v.node(2)
    assert r["log_len"] == 1 and r["entries_is_seq"] == 1 and r["commit_index"] == 3
    assert r["fault"] == 0
    d = r["deadline"]
    v.step(d)          # the timeout fires: last-entry (nth (x) 2) throws
    r = v.node(2)
    assert r["fault"] == 1 and r["role"] == ROLE["follwer"] and r["current_term"] == 2
    assert v.counters()["halt_ioobe"] == 1


def kat_cce(view_of):
    """A LazySeq log reaching leadership: entries-from's subvec throws CCE (log.clj:53)."""
    nodes = {1: node("candidate", term=3, voted_for=1, votes=[1], log=[E1], commit=1, is_seq=1),
             2: node(), 3: node()}
    q = {(1, 1): [msg("vote-response", 0, term=1, id=2, vote_granted=True)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(1)
    r = v.node(1)
    # halted with the pre-event state: still a candidate with the old votes
    assert r["fault"] == 3 and r["role"] == ROLE["candidate"] and r["votes"] == 1 << 1
    assert v.counters()["halt_cce"] == 1 and v.counters()["sent"] == 0


def kat_npe(view_of):
    """append-response failure with nil leader-state: (dec nil) throws NPE (core.clj:146)."""
    nodes = {1: node("follower", term=2), 2: node()}
    q = {(1, 1): [msg("append-response", 0, term=2, id=2, success=False)]}
    v = view_of(Scenario(2, nodes, q))
    v.step(1)
    assert v.node(1)["fault"] == 2 and v.counters()["halt_npe"] == 1


def kat_partial_leader_state(view_of):
    """append-response success on a non-leader creates a partial leader-state (core.clj:147-149)."""
    nodes = {1: node("follower", term=2), 2: node(), 3: node()}
    q = {(1, 1): [msg("append-response", 0, term=2, id=3, success=True, commit=4, log_index=6)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(1)
    r = v.node(1)
    assert r["ls_present"] == 1 and r["ls_keys"] == 1 << 3 and r["role"] == ROLE["follower"]
    assert r["next_index"][2] == 6 and r["match_index"][2] == 4


def kat_stale_step_down(view_of):
    """vote-response with a higher term: :follwer, leader-state and leader-id kept (core.clj:130)."""
    ls = {2: (1, 0), 3: (1, 0)}
    nodes = {1: node("leader", term=2, leader_id=1, ls=ls), 2: node(), 3: node()}
    q = {(1, 1): [msg("vote-response", 0, term=5, id=2, vote_granted=False)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(1)
    r = v.node(1)
    assert (r["role"], r["current_term"], r["leader_id"], r["ls_present"]) == \
        (ROLE["follwer"], 5, 1, 1)
    # append-response with a higher term: leader->follower clears both (core.clj:86-89,145)
    nodes[1] = node("leader", term=2, leader_id=1, ls=ls, voted_for=0)
    q = {(1, 1): [msg("append-response", 0, term=4, id=3, success=False)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(1)
    r = v.node(1)
    assert (r["role"], r["current_term"], r["leader_id"], r["ls_present"]) == \
        (ROLE["follower"], 4, 0, 0)


def kat_two_leaders_one_term(view_of):
    """Leader A (term 2, voted-for nil, core.clj:82); a delayed candidate B wins term 2 too."""
    nodes = {1: node("leader", term=2, leader_id=1, ls={2: (1, 0), 3: (1, 0)}, last_led=2),
             2: node("candidate", term=2, voted_for=2, votes=[2]),
             3: node("follwer", term=2, leader_id=1)}
    q = {(2, 1): [msg("vote-response", 0, term=2, id=3, vote_granted=True)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(1)
    assert v.node(2)["role"] == ROLE["leader"] and v.node(1)["role"] == ROLE["leader"]
    c = v.counters()
    assert c["viol_election"] == 1 and c["leaders"] == 1


def kat_vote_rules(view_of):
    """request-vote-handler (core.clj:91-103): lower term, existing vote, or log mismatch refuse."""
    nodes = {1: node(term=3, log=[E1], commit=1), 2: node(), 3: node()}
    q = {(1, 0): [msg("request-vote", 0, term=2, candidate_id=2, last_log_index=0,
                      last_log_term=None),
                  msg("request-vote", 0, term=4, candidate_id=3, last_log_index=1,
                      last_log_term=(9, 9)),
                  msg("request-vote", 0, term=4, candidate_id=3, last_log_index=1,
                      last_log_term=E1),
                  msg("request-vote", 0, term=5, candidate_id=2, last_log_index=0,
                      last_log_term=None),
                  msg("request-vote", 0, term=5, candidate_id=2, last_log_index=4,
                      last_log_term=None)]}
    v = view_of(Scenario(3, nodes, q))
    v.step(2)
    assert v.node(1)["voted_for"] == 0            # stale term, then mismatching entry
    v.step(1)
    r = v.node(1)
    assert r["voted_for"] == 3 and r["current_term"] == 3   # granted, term unchanged
    v.step(1)
    assert v.node(1)["voted_for"] == 3            # already voted
    v.step(1)
    assert v.node(1)["fault"] == 1                # last-log-index 4 > count: nth throws


def kat_variant_no_log_check(view_of):
    """VOTE_NO_LOG_CHECK skips compare-prev? (core.clj:96,99): no throw, vote granted."""
    nodes = {1: node(term=1), 2: node()}
    q = {(1, 0): [msg("request-vote", 0, term=2, candidate_id=2, last_log_index=4,
                      last_log_term=None)]}
    scn = Scenario(2, nodes, q, variant_flags=1)
    v = view_of(scn)
    v.step(1)
    assert v.node(1)["fault"] == 0 and v.node(1)["voted_for"] == 2


def kat_client_set(view_of):
    """client-set (core.clj:151-160): leader appends (term, val); others only redirect."""
    nodes = {1: node("leader", term=4, leader_id=1, ls={2: (1, 0)}), 2: node(term=4)}
    q = {(1, 0): [msg("client-set", 0, command=77)], (2, 0): [msg("client-set", 0, command=5)]}
    v = view_of(Scenario(2, nodes, q))
    v.step(1)
    assert v.log(1) == [(4, 77)] and v.log(2) == []
    assert v.node(2)["deadline"] >= 5000          # the event still re-arms the timer


def kat_client_abandoned_without_redirects(view_of):
    """client_redirects = 0: a redirect ends the command (counted as abandoned, nothing re-sent)."""
    nodes = {1: node("leader", term=4, leader_id=1, ls={2: (1, 0)}), 2: node(term=4, leader_id=1)}
    q = {(2, 0): [msg("client-set", 0, command=5)]}
    v = view_of(Scenario(2, nodes, q))
    v.step(3)
    c = v.counters()
    assert c["client_abandoned"] == 1 and c["redirects"] == 0 and v.log(1) == []


def kat_redirect_to_leader(view_of):
    """redirect-client (server.clj:62-63) to the :leader-id (core.clj:155), followed by the client:
    the command reaches the leader one tick later and is appended (core.clj:156-160); a node with
    a nil :leader-id redirects to (rand-nth cluster) (core.clj:154), drawn from w2 of its EVENT
    draw (SIM_SPEC D15)."""
    nodes = {1: node("leader", term=4, leader_id=1, ls={2: (1, 0), 3: (1, 0)}),
             2: node("follwer", term=4, leader_id=1), 3: node(term=4)}
    q = {(2, 0): [msg("client-set", 0, command=5)], (3, 0): [msg("client-set", 0, command=6)]}
    v = view_of(Scenario(3, nodes, q, client_redirects=2))
    w = pyref.philox((0, 3 | pyref.EVENT << 8, 0, 0), (42, 0))
    target = [1, 2][(w[2] * 2) >> 32]
    v.step(1)                                     # t0: both redirect (no state change)
    assert v.log(1) == [] and v.node(2)["log_len"] == 0
    assert v.node(2)["deadline"] >= 5000          # D4: the redirect still re-arms the timer
    v.step(1)                                     # t1: the leader appends node 2's redirect
    assert v.log(1) == [(4, 5)]
    v.step(2 if target == 1 else 3)
    assert v.log(1) == [(4, 5), (4, 6)]
    c = v.counters()
    assert c["redirects"] == (2 if target == 1 else 3) and c["client_abandoned"] == 0
    assert c["ev_cs"] == (4 if target == 1 else 5) and c["sent"] == 0


def kat_redirect_to_self(view_of):
    """A stepped-down leader keeps its own :leader-id (candidate->follower, core.clj:75-78,130), so
    redirect-client points the client back at it; each hop is an event until the hops run out."""
    nodes = {1: node("follwer", term=5, leader_id=1, ls={2: (1, 0)}), 2: node(term=5)}
    q = {(1, 0): [msg("client-set", 0, command=9)]}
    v = view_of(Scenario(2, nodes, q, client_redirects=2))
    v.step(4)
    c = v.counters()
    assert (c["ev_cs"], c["redirects"], c["client_abandoned"]) == (3, 2, 1)
    assert v.log(1) == [] and v.node(1)["req_count"] == 0


CHAN = "#<ManyToManyChannel clojure.core.async.impl.channels.ManyToManyChannel@%x>"


def kat_printed_trace(view_of):
    """What `wait` prints (core.clj:182-186) over a 3-node first election: the pre-handler node
    map in init-node key order (core.clj:31-38), request bodies in the sender's literal order plus
    :type and :resp-chan (core.clj:51-54,62-67; server.clj:14-21), replies {:term :id :type ..}
    carrying the voter's own, never-updated term (core.clj:94,100)."""
    nodes = {i: node(deadline=BIG) for i in range(1, 4)}
    nodes[3] = node(deadline=0)
    v = view_of(Scenario(3, nodes))
    v.step(4)   # t0 timeout, t1 votes, t2 first grant -> leader (2 of 3), t3 second grant + AEs
    rv = ("{:term 2, :candidate-id 3, :last-log-index 0, :last-log-term nil, "
          ":type :request-vote, :resp-chan " + CHAN % 0 + "}")
    assert v.edn(3) == (
        "; Node\n"
        "{:id 3, :state :follower, :current-term 1, :voted-for nil, :leader-id nil, "
        ":leader-state nil, :votes #{}}\n"
        "; Message\nnil\n\n"
        "; Node\n"
        "{:id 3, :state :candidate, :current-term 2, :voted-for 3, :leader-id nil, "
        ":leader-state nil, :votes #{3}}\n"
        "; Message\n{:term 1, :id 1, :type :vote-response, :vote-granted true}\n\n"
        "; Node\n"
        "{:id 3, :state :leader, :current-term 2, :voted-for nil, :leader-id 3, "
        ":leader-state {:next-index {1 1, 2 1}, :match-index {1 0, 2 0}}, :votes #{}}\n"
        "; Message\n{:term 1, :id 2, :type :vote-response, :vote-granted true}\n\n")
    assert v.edn(1) == (
        "; Node\n"
        "{:id 1, :state :follower, :current-term 1, :voted-for nil, :leader-id nil, "
        ":leader-state nil, :votes #{}}\n"
        "; Message\n" + rv + "\n\n"
        "; Node\n"
        "{:id 1, :state :follower, :current-term 1, :voted-for 3, :leader-id nil, "
        ":leader-state nil, :votes #{}}\n"
        "; Message\n"
        "{:term 2, :leader-id 3, :leader-commit 0, :prev-log-index 0, :prev-log-term nil, "
        ":entries [], :type :append-entries, :resp-chan " + CHAN % 1 + "}\n\n")


def kat_printed_entries(view_of):
    """An append-entries prints its :entries (log.clj:67 shape) and its prev-log-term entry."""
    ls = {2: (1, 0)}
    nodes = {1: node("leader", term=2, leader_id=1, ls=ls, log=[E1, E2, E3], deadline=0,
                     last_led=2),
             2: node("follwer", term=2, leader_id=1, deadline=BIG)}
    v = view_of(Scenario(2, nodes))
    v.step(2)
    assert v.edn(2).split("\n")[3] == (
        "{:term 2, :leader-id 1, :leader-commit 0, :prev-log-index 0, "
        ":prev-log-term {:term 2, :val 10}, :entries [{:term 2, :val 20} {:term 2, :val 30}], "
        ":type :append-entries, :resp-chan " + CHAN % 0 + "}")


# ================================================================ F4 Spec-Raft (SIM_SPEC §8)
# Not reference behaviour: Raft Figure 2 (Ongaro & Ousterhout 2014), the correct-protocol control.
SPEC = 2


def kat_spec_first_election(view_of):
    """Voters adopt the candidate's term (Figure 2 "all servers"), keep voted-for, followers
    become :follower (not :follwer) and the leader keeps voted-for; next = last log index + 1."""
    nodes = {i: node(deadline=BIG) for i in range(1, 6)}
    nodes[3] = node(deadline=0)
    v = view_of(Scenario(5, nodes, variant_flags=SPEC))
    v.step(1)
    assert (v.node(3)["role"], v.node(3)["current_term"], v.node(3)["voted_for"]) == \
        (ROLE["candidate"], 2, 3)
    v.step(1)
    for i in (1, 2, 4, 5):
        r = v.node(i)
        assert (r["role"], r["current_term"], r["voted_for"]) == (ROLE["follower"], 2, 3), r
    v.step(2)                                    # t2 first grant, t3 second grant: 3 of 5
    a = v.node(3)
    assert (a["role"], a["votes"], a["voted_for"], a["leader_id"]) == (ROLE["leader"], 0, 3, 3)
    assert a["next_index"] == [1, 1, 0, 1, 1] and a["match_index"] == [0] * 5
    v.step(1)
    for i in (1, 2, 4, 5):
        r = v.node(i)
        assert (r["role"], r["current_term"], r["voted_for"], r["leader_id"]) == \
            (ROLE["follower"], 2, 3, 3), r
    v.step(5)
    a = v.node(3)
    assert a["next_index"] == [1, 1, 0, 1, 1] and a["commit_index"] == 0
    c = v.counters()
    assert c["leaders"] == 1 and c["ev_vr"] == 4 and c["ev_ar"] == 4 and c["ev_ae"] == 4


def kat_spec_replication(view_of):
    """The whole suffix ships once, the leader commits by majority match, followers learn the
    commit from the next heartbeat, and nothing is duplicated."""
    nodes = {1: node("leader", term=2, voted_for=1, leader_id=1, ls={2: (1, 0), 3: (1, 0)},
                     log=[E1, E2, E3], deadline=0, last_led=2),
             2: node("follower", term=2, voted_for=1, leader_id=1),
             3: node("follower", term=2, voted_for=1, leader_id=1)}
    v = view_of(Scenario(3, nodes, variant_flags=SPEC))
    v.step(2)                                    # t0 heartbeat, t1 followers append all three
    assert v.log(2) == [E1, E2, E3] and v.log(3) == [E1, E2, E3]
    assert v.node(2)["commit_index"] == 0        # leader-commit was 0
    v.step(1)                                    # t2 reply from 2: match {3, 3, 0} -> commit 3
    a = v.node(1)
    assert a["commit_index"] == 3 and v.commit_stream(1) == [10, 20, 30]
    v.step(1)
    a = v.node(1)
    assert a["next_index"] == [0, 4, 4] and a["match_index"] == [0, 3, 3]
    v.step(3002)                                 # heartbeat at 3003 (hb after t3), lands 3004
    for i in (2, 3):
        assert v.log(i) == [E1, E2, E3] and v.node(i)["commit_index"] == 3
        assert v.commit_stream(i) == [10, 20, 30]
    c = v.counters()
    assert c["viol_log"] == 0 and c["entries_appended"] == 6 and c["entries_applied"] == 9


F = (3, 40)


def kat_spec_truncate_on_conflict(view_of):
    """A conflicting suffix is truncated at the first term mismatch and replaced; a duplicate or a
    shorter consistent AppendEntries never shortens the log."""
    nodes = {1: node("leader", term=3, voted_for=1, leader_id=1, ls={2: (2, 0), 3: (3, 0)},
                     log=[E1, F], commit=1, deadline=0, last_led=3),
             2: node("follower", term=3, leader_id=1, log=[E1, (2, 99), (2, 98)], commit=1),
             3: node("follower", term=3, leader_id=1, log=[E1, F])}
    q = {(2, 0): [msg("append-entries", 1, term=3, leader_id=1, leader_commit=1,
                      prev_log_index=1, prev_log_term=E1, entries=[F])],
         (3, 0): [msg("append-entries", 1, term=3, leader_id=1, leader_commit=1,
                      prev_log_index=1, prev_log_term=E1, entries=[])]}
    v = view_of(Scenario(3, nodes, q, variant_flags=SPEC))
    v.step(1)                                    # t0 heartbeat: prev 1 (E1) + [F] to node 2
    v.step(1)                                    # t1: the queued duplicates (arrival 1) first
    assert v.log(2) == [E1, F] and v.node(2)["log_len"] == 2   # (2,99),(2,98) truncated
    assert v.log(3) == [E1, F]                   # shorter AE: log kept
    v.step(1)                                    # t2: the heartbeat's copies: idempotent
    assert v.log(2) == [E1, F] and v.log(3) == [E1, F]
    assert v.node(2)["commit_index"] == 1 and v.node(2)["fault"] == 0


def kat_spec_commit_rule(view_of):
    """Figure 8: a majority-replicated entry of an older term is not committed by counting; an
    entry of the leader's own term commits it indirectly."""
    nodes = {1: node("leader", term=4, voted_for=1, leader_id=1, ls={2: (3, 0), 3: (3, 0)},
                     log=[(2, 10), (2, 20)], last_led=4),
             2: node("follower", term=4, leader_id=1, log=[(2, 10), (2, 20)]), 3: node(term=4)}
    q = {(1, 1): [msg("append-response", 0, term=4, id=2, success=True, commit=0, log_index=2),
                  msg("append-response", 2, term=4, id=2, success=True, commit=0, log_index=3)],
         (1, 0): [msg("client-set", 1, command=77)]}
    v = view_of(Scenario(3, nodes, q, variant_flags=SPEC))
    v.step(1)
    assert v.node(1)["commit_index"] == 0 and v.node(1)["match_index"] == [0, 2, 0]
    v.step(1)
    assert v.log(1) == [(2, 10), (2, 20), (4, 77)]
    v.step(1)
    a = v.node(1)
    assert a["commit_index"] == 3 and v.commit_stream(1) == [10, 20, 77]
    assert a["next_index"][1] == 4 and a["match_index"][1] == 3


def kat_spec_vote_rules(view_of):
    """Up-to-date check (last term, then length), one vote per term, term update on any RPC."""
    def rv(term, cand, idx, last):
        return msg("request-vote", 0, term=term, candidate_id=cand, last_log_index=idx,
                   last_log_term=last)
    for flags in (SPEC, SPEC | 1):
        nodes = {1: node(term=3, log=[(3, 1)]), 2: node(term=3), 3: node(term=3)}
        q = {(1, 0): [rv(3, 2, 5, (2, 9)), rv(3, 2, 0, None), rv(3, 3, 1, (3, 5)),
                      rv(3, 2, 9, (4, 0)), rv(3, 3, 1, (3, 5)), rv(5, 2, 0, None)]}
        v = view_of(Scenario(3, nodes, q, variant_flags=flags))
        v.step(1)                                # older last term: refused (granted without check)
        assert v.node(1)["voted_for"] == (0 if flags == SPEC else 2)
        if flags != SPEC:
            continue
        v.step(1)
        assert v.node(1)["voted_for"] == 0       # empty log is behind
        v.step(1)
        assert v.node(1)["voted_for"] == 3       # same last term, index >= 1: granted
        v.step(1)
        assert v.node(1)["voted_for"] == 3       # one vote per term
        v.step(1)
        assert v.node(1)["voted_for"] == 3       # the same candidate again
        v.step(1)
        r = v.node(1)
        assert (r["current_term"], r["voted_for"], r["role"]) == (5, 0, ROLE["follower"])
        assert r["fault"] == 0


def kat_spec_timers(view_of):
    """Raft §5.2 timers (SIM_SPEC §8): a leader heartbeats every hb ticks whatever it handles; a
    follower's election timer moves only for AppendEntries from the current leader, a granted
    vote or its own timeout -- not for client-sets, redirects or stale messages."""
    nodes = {1: node("leader", term=3, voted_for=1, leader_id=1, ls={2: (1, 0), 3: (1, 0)},
                     deadline=10, last_led=3),
             2: node("follower", term=3, leader_id=1, deadline=500),
             3: node("follower", term=3, leader_id=1, deadline=BIG)}
    q = {(1, 0): [msg("client-set", 0, command=7)],
         (2, 0): [msg("client-set", 0, command=8),
                  msg("request-vote", 1, term=2, candidate_id=3, last_log_index=0,
                      last_log_term=None)]}
    v = view_of(Scenario(3, nodes, q, variant_flags=SPEC, client_redirects=1))
    v.step(1)                                    # t0: leader appends, follower 2 redirects
    assert v.node(1)["deadline"] == 10 and v.node(2)["deadline"] == 500
    v.step(2)                                    # t1: stale RV refused; t2: redirected set
    assert v.node(2)["deadline"] == 500 and v.log(1) == [(3, 7), (3, 8)]
    assert v.node(1)["deadline"] == 10
    v.step(8)                                    # t10: heartbeat -> next one at 3010
    assert v.node(1)["deadline"] == 3010
    v.step(1)                                    # t11: AppendEntries re-arms the followers
    assert v.node(2)["deadline"] >= 11 + 5000 and v.node(3)["deadline"] >= 11 + 5000


SPEC_ALL = [kat_spec_timers, kat_spec_first_election, kat_spec_replication, kat_spec_truncate_on_conflict,
            kat_spec_commit_rule, kat_spec_vote_rules]

ALL = [kat_majority, kat_first_election, kat_duplication, kat_truncate_crash, kat_cce, kat_npe,
       kat_partial_leader_state, kat_stale_step_down, kat_two_leaders_one_term, kat_vote_rules,
       kat_variant_no_log_check, kat_client_set, kat_client_abandoned_without_redirects,
       kat_redirect_to_leader, kat_redirect_to_self, kat_printed_trace, kat_printed_entries,
       *SPEC_ALL]
