"""Deterministic discrete-time counterpart of the reference's Raft test harness
(src/raft/config.go) driving one Raft group through the engine's C ABI —
config #1 of BASELINE.json ("src/raft 3-peer single group via labrpc harness,
go test -run 2B"). Test infrastructure.

Mapping to the reference:
  * time advances in 10 ms ticks; heartbeats every 90 ms (raft.go:42-44),
    randomized election timeouts 300-600 ms (raft.go:46-50), seeded;
  * labrpc's connect/disconnect (labrpc.go:349-364, config.go:366-409): a
    message is delivered iff both endpoints are connected;
  * a server's timer fires StartElection (raft.go:106-125 ->
    raft_election.go:4-51); RequestVotes are delivered in candidate order,
    replies tallied in voter order; a new leader heartbeats at once (:39-40);
  * a leader's heartbeat/append (raft_append_entry.go:4-65) is one batched
    gather -> handle -> reply fold through the ABI, repeated while a
    follower still needs entries (raft.go:127-150);
  * election-timer resets at raft_append_entry.go:71,121 and
    raft_election.go:72;
  * the applier (raft.go:153-203) feeds cfg.logs with the same checks as
    config.go:144-163 (same index => same command; in-order apply);
  * one(), checkOneLeader(), nCommitted() follow config.go:569-622, 438-468,
    502-524;
  * persistence (2C): after every batch of engine calls the replicas the
    engine marked persist_dirty are saved to a per-server Persister
    (multiraft_amd.persister, persister.go); crash1 / start1
    (config.go:112-142, 283-340) kill a server and restart it with Make +
    readPersist from its last persisted bytes (mraft_restore). A replica
    whose state changed without a persist mark would lose that change here.
Commands never enter the engine: the harness keeps each server's commands
index-aligned with its log (the host side of the boundary, include/mraft.h).
"""
from __future__ import annotations

import numpy as np

from multiraft_amd._abi import (AE_RESULT, F_BECAME_LEADER, F_NEED_MORE, F_STEPPED_DOWN, FOLLOWER,
                                LEADER, RV_ARGS, RV_RESULT)
from multiraft_amd.engine import new_state
from multiraft_amd.persister import Persister, flush_persist, restart

TICK_MS = 10
HEARTBEAT = 9          # ticks
ELECTION = (30, 60)    # ticks
RAFT_ELECTION_TIMEOUT = 100  # ticks = 1 s (test_test.go:22)


class HarnessFailure(AssertionError):
    pass


class Cluster:
    """One Raft group of P servers (G = 1) over an engine-like backend."""

    def __init__(self, make_backend, P: int, L: int = 512, seed: int = 1):
        self.P, self.L = P, L
        st = new_state(1, P, L)
        self.eng = make_backend(1, P, L, st)
        self.rng = np.random.default_rng(seed)
        self.now = 0
        self.connected = [True] * P
        self.elec = [self._etimeout() for _ in range(P)]
        self.hb = [0] * P
        self.cmds = [dict() for _ in range(P)]      # host command mirror: index -> cmd
        self.logs = [dict() for _ in range(P)]      # cfg.logs: applied index -> cmd
        self.max_index = 0
        self.rpcs = 0
        self.alive = [True] * P                     # cfg.rafts[i] != nil
        self.persister = Persister(P)               # cfg.saved
        self.saved_cmds = [dict() for _ in range(P)]  # commands persisted beside the raft state
        self.st = self.eng.store_state()

    # ---- helpers ---------------------------------------------------------
    def _etimeout(self):
        return self.now + int(self.rng.integers(ELECTION[0], ELECTION[1]))

    def _refresh(self):
        self.st = self.eng.store_state()

    def role(self, p):
        return int(self.st["state"][p])

    def term(self, p):
        return int(self.st["current_term"][p])

    def _link(self, a, b):
        return self.connected[a] and self.connected[b] and self.alive[a] and self.alive[b]

    def _flush(self):
        """The persist() call sites of the last batch, saved (persister.go)."""
        for p in flush_persist(self.eng, self.persister):
            self.saved_cmds[int(p)] = dict(self.cmds[int(p)])

    def crash1(self, p):
        """config.go:112-142: disconnect, kill; the persisted bytes survive."""
        self.disconnect(p)
        self.alive[p] = False

    def start1(self, p):
        """config.go:283-340: crash1, then Make + readPersist from the saved
        state; the server stays disconnected until connect()."""
        self.crash1(p)
        err = restart(self.eng, self.persister, [p])
        assert not err.any(), err
        self.cmds[p] = dict(self.saved_cmds[p])
        self.alive[p] = True
        self.elec[p] = self._etimeout()
        self.hb[p] = 0
        self._refresh()

    def connect(self, p):
        self.connected[p] = True

    def disconnect(self, p):
        self.connected[p] = False

    # ---- Raft API mirror --------------------------------------------------
    def start(self, p, cmd):
        """Raft.Start (raft.go:90-104) on server p."""
        if not self.alive[p]:
            return -1, -1, False
        idx, term, isl, err = self.eng.start(np.array([p], np.int32))
        assert not err.any(), err
        if not isl[0]:
            return -1, -1, False
        self.cmds[p][int(idx[0])] = cmd
        self._flush()
        self._refresh()
        self._replicate([p])  # BroadcastAppend(Append)
        self._flush()
        return int(idx[0]), int(term[0]), True

    def get_state(self, p):
        """GetState (raft.go:237-246)."""
        return self.term(p), self.role(p) == LEADER

    # ---- one tick ---------------------------------------------------------
    def step(self):
        self.now += 1
        self._refresh()
        cands = []
        for p in range(self.P):
            if self.alive[p] and self.now >= self.elec[p]:
                self.elec[p] = self._etimeout()
                if self.role(p) != LEADER:
                    cands.append(p)
        if cands:
            self._election(cands)
        self._refresh()
        leaders = [p for p in range(self.P)
                   if self.alive[p] and self.role(p) == LEADER and self.now >= self.hb[p]]
        if leaders:
            self._replicate(leaders)
        self._flush()
        self._apply()

    def advance(self, ticks):
        for _ in range(ticks):
            self.step()

    # ---- elections --------------------------------------------------------
    def _election(self, cands):
        args, err = self.eng.start_election(np.array(cands, np.int32))
        assert not err.any(), err
        # RequestVote deliveries, one round per candidate (arrival order).
        results = {c: [] for c in cands}
        for ci, c in enumerate(cands):
            items, peers = [], []
            for v in range(self.P):
                if v == c or not self._link(c, v):
                    continue
                a = args[ci]
                items.append((v, a["candidate_id"], a["term"], a["last_log_index"], a["last_log_term"]))
                peers.append(v)
            if not items:
                continue
            rv = np.array(items, dtype=RV_ARGS)
            self.rpcs += len(items)
            rep, rerr = self.eng.handle_request_vote(rv)
            assert not rerr.any(), rerr
            for v, r in zip(peers, rep):
                if r["vote_granted"]:
                    self.elec[v] = self._etimeout()           # raft_election.go:72
                results[c].append((c, v, int(args[ci]["term"]), int(r["term"]), int(r["vote_granted"])))
        items, seg = [], [0]
        for c in cands:
            items += results[c]
            if results[c]:
                seg.append(len(items))
        if not items:
            return
        flags, ferr = self.eng.process_vote_replies(np.array(items, dtype=RV_RESULT),
                                                    np.array(seg, np.int64))
        assert not ferr.any(), ferr
        new_leaders = sorted({items[i][0] for i in range(len(items)) if flags[i] & F_BECAME_LEADER})
        for i in range(len(items)):
            if flags[i] & F_STEPPED_DOWN:
                pass  # the tally's step-down resets no timer in the reference
        if new_leaders:
            self._refresh()
            self._replicate(new_leaders)                      # BroadcastAppend(HeartBeat)

    # ---- replication -------------------------------------------------------
    def _replicate(self, leaders, max_rounds=16):
        for _ in range(max_rounds):
            self._refresh()
            slots, peers = [], []
            for ld in leaders:
                if self.role(ld) != LEADER:
                    continue
                self.hb[ld] = self.now + HEARTBEAT
                for p in range(self.P):
                    if p != ld:
                        slots.append(ld)
                        peers.append(p)
            if not slots:
                return
            args, gerr = self.eng.gather_append_args(np.array(slots, np.int32), np.array(peers, np.int32))
            deliver = [i for i in range(len(slots))
                       if gerr[i] == 0 and self._link(slots[i], peers[i])]
            if not deliver:
                return
            # AppendEntries to distinct followers per call (one round per leader).
            results = []
            by_leader = {}
            for i in deliver:
                by_leader.setdefault(slots[i], []).append(i)
            for ld, idxs in by_leader.items():
                a = args[idxs]
                self.rpcs += len(idxs)
                rep, herr = self.eng.handle_append_entries(a, None)
                assert not herr.any(), herr
                for j, i in enumerate(idxs):
                    f = peers[i]
                    r = rep[j]
                    if not (r["term"] > a[j]["term"]):              # not the stale path:
                        self.elec[f] = self._etimeout()             # :121 timer reset
                    if r["success"]:
                        prev, n = int(a[j]["prev_log_index"]), int(a[j]["n_entries"])
                        for x in range(prev + 1, prev + n + 1):     # host command mirror
                            self.cmds[f][x] = self.cmds[ld].get(x)
                    results.append((ld, f, int(a[j]["term"]), int(a[j]["prev_log_index"]),
                                    int(a[j]["n_entries"]), int(r["term"]), int(r["success"]),
                                    int(r["conflict_index"])))
            results.sort(key=lambda t: (t[0], t[1]))
            seg, cur = [0], None
            for i, t in enumerate(results):
                if cur is not None and t[0] != cur:
                    seg.append(i)
                cur = t[0]
            seg.append(len(results))
            flags, ferr = self.eng.process_append_replies(np.array(results, dtype=AE_RESULT),
                                                          np.array(seg, np.int64))
            assert not ferr.any(), ferr
            more = False
            for i, t in enumerate(results):
                if flags[i] & F_STEPPED_DOWN:
                    self.elec[t[0]] = self._etimeout()              # :71 timer reset
                if flags[i] & F_NEED_MORE:
                    more = True
            self._apply()
            if not more:
                return

    # ---- applier + cfg.logs checks (config.go:144-163) --------------------
    def _apply(self):
        fr, to = self.eng.collect_apply()
        for p in range(self.P):
            if not self.alive[p]:
                continue
            for i in range(int(fr[p]), int(to[p]) + 1):
                cmd = self.cmds[p].get(i)
                for q in range(self.P):
                    if i in self.logs[q] and self.logs[q][i] != cmd:
                        raise HarnessFailure(f"commit index={i} server={p} {cmd} != server={q} {self.logs[q][i]}")
                if i > 1 and (i - 1) not in self.logs[p]:
                    raise HarnessFailure(f"server {p} apply out of order {i}")
                self.logs[p][i] = cmd
                self.max_index = max(self.max_index, i)

    # ---- config.go helpers -------------------------------------------------
    def n_committed(self, index):
        count, cmd = 0, None
        for p in range(self.P):
            if index in self.logs[p]:
                c = self.logs[p][index]
                if count > 0 and cmd != c:
                    raise HarnessFailure(f"committed values do not match: index {index}")
                count, cmd = count + 1, c
        return count, cmd

    def check_one_leader(self):
        for _ in range(10):
            self.advance(int(self.rng.integers(45, 56)))
            self._refresh()
            leaders = {}
            for p in range(self.P):
                if self.connected[p] and self.alive[p] and self.role(p) == LEADER:
                    leaders.setdefault(self.term(p), []).append(p)
            last = -1
            for t, ls in leaders.items():
                if len(ls) > 1:
                    raise HarnessFailure(f"term {t} has {len(ls)} (>1) leaders")
                last = max(last, t)
            if leaders:
                return leaders[last][0]
        raise HarnessFailure("expected one leader, got none")

    def check_terms(self):
        term = -1
        for p in range(self.P):
            if self.connected[p]:
                t, _ = self.get_state(p)
                if term == -1:
                    term = t
                elif term != t:
                    raise HarnessFailure("servers disagree on term")
        return term

    def one(self, cmd, expected, retry):
        t0 = self.now
        starts = 0
        while self.now - t0 < 1000:
            index = -1
            for _ in range(self.P):
                starts = (starts + 1) % self.P
                if self.connected[starts] and self.alive[starts]:
                    idx, _, ok = self.start(starts, cmd)
                    if ok:
                        index = idx
                        break
            if index != -1:
                t1 = self.now
                while self.now - t1 < 200:
                    nd, c = self.n_committed(index)
                    if nd > 0 and nd >= expected and c == cmd:
                        return index
                    self.advance(2)
                if not retry:
                    raise HarnessFailure(f"one({cmd}) failed to reach agreement")
            else:
                self.advance(5)
        raise HarnessFailure(f"one({cmd}) failed to reach agreement")


# ---------------------------------------------------------------------------
# Scenarios: the assertions of src/raft/test_test.go
# ---------------------------------------------------------------------------

def initial_election_2a(mk, seed=1):                 # test_test.go:24-53
    cfg = Cluster(mk, 3, seed=seed)
    cfg.check_one_leader()
    cfg.advance(5)
    t1 = cfg.check_terms()
    assert t1 >= 1, "term is 0 after election"
    cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    cfg.check_terms()  # the reference only warns if the term changed (:45-47)
    cfg.check_one_leader()


def re_election_2a(mk, seed=2):                      # test_test.go:55-93
    cfg = Cluster(mk, 3, seed=seed)
    l1 = cfg.check_one_leader()
    cfg.disconnect(l1)
    cfg.check_one_leader()
    cfg.connect(l1)
    l2 = cfg.check_one_leader()
    cfg.disconnect(l2)
    cfg.disconnect((l2 + 1) % 3)
    cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    cfg._refresh()
    assert not any(cfg.connected[p] and cfg.role(p) == LEADER for p in range(3)), "leader without majority"
    cfg.connect((l2 + 1) % 3)
    cfg.check_one_leader()
    cfg.connect(l2)
    cfg.check_one_leader()


def basic_agree_2b(mk, seed=3):                      # test_test.go:128-153
    cfg = Cluster(mk, 3, seed=seed)
    for index in range(1, 4):
        nd, _ = cfg.n_committed(index)
        assert nd == 0, "some have committed before Start()"
        x = cfg.one(index * 100, 3, False)
        assert x == index, f"got index {x} but expected {index}"


def fail_agree_2b(mk, seed=4):                       # test_test.go:279-311
    cfg = Cluster(mk, 3, seed=seed)
    cfg.one(101, 3, False)
    leader = cfg.check_one_leader()
    cfg.disconnect((leader + 1) % 3)
    cfg.one(102, 2, False)
    cfg.one(103, 2, False)
    cfg.advance(RAFT_ELECTION_TIMEOUT)
    cfg.one(104, 2, False)
    cfg.one(105, 2, False)
    cfg.connect((leader + 1) % 3)
    cfg.one(106, 3, True)
    cfg.advance(RAFT_ELECTION_TIMEOUT)
    cfg.one(107, 3, True)


def fail_no_agree_2b(mk, seed=5):                    # test_test.go:313-362
    cfg = Cluster(mk, 5, seed=seed)
    cfg.one(10, 5, False)
    leader = cfg.check_one_leader()
    for k in (1, 2, 3):
        cfg.disconnect((leader + k) % 5)
    index, _, ok = cfg.start(leader, 20)
    assert ok, "leader rejected Start()"
    assert index == 2, f"expected index 2, got {index}"
    cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    n, _ = cfg.n_committed(index)
    assert n == 0, f"{n} committed but no majority"
    for k in (1, 2, 3):
        cfg.connect((leader + k) % 5)
    leader2 = cfg.check_one_leader()
    index2, _, ok2 = cfg.start(leader2, 30)
    assert ok2, "leader2 rejected Start()"
    assert 2 <= index2 <= 3, f"unexpected index {index2}"
    cfg.one(1000, 5, True)


def rejoin_2b(mk, seed=6):                           # test_test.go:465-501
    cfg = Cluster(mk, 3, seed=seed)
    cfg.one(101, 3, True)
    leader1 = cfg.check_one_leader()
    cfg.disconnect(leader1)
    cfg.start(leader1, 102)
    cfg.start(leader1, 103)
    cfg.start(leader1, 104)
    cfg.one(103, 2, True)
    leader2 = cfg.check_one_leader()
    cfg.disconnect(leader2)
    cfg.connect(leader1)
    cfg.one(104, 2, True)
    cfg.connect(leader2)
    cfg.one(105, 3, True)


def backup_2b(mk, seed=7):                           # test_test.go:503-573
    rng = np.random.default_rng(seed)
    cmd = lambda: int(rng.integers(1, 1 << 30))  # noqa: E731
    cfg = Cluster(mk, 5, seed=seed)
    cfg.one(cmd(), 5, True)
    leader1 = cfg.check_one_leader()
    for k in (2, 3, 4):
        cfg.disconnect((leader1 + k) % 5)
    for _ in range(50):
        cfg.start(leader1, cmd())
    cfg.advance(RAFT_ELECTION_TIMEOUT // 2)
    cfg.disconnect((leader1 + 0) % 5)
    cfg.disconnect((leader1 + 1) % 5)
    for k in (2, 3, 4):
        cfg.connect((leader1 + k) % 5)
    for _ in range(50):
        cfg.one(cmd(), 3, True)
    leader2 = cfg.check_one_leader()
    other = (leader1 + 2) % 5
    if leader2 == other:
        other = (leader2 + 1) % 5
    cfg.disconnect(other)
    for _ in range(50):
        cfg.start(leader2, cmd())
    cfg.advance(RAFT_ELECTION_TIMEOUT // 2)
    for i in range(5):
        cfg.disconnect(i)
    cfg.connect((leader1 + 0) % 5)
    cfg.connect((leader1 + 1) % 5)
    cfg.connect(other)
    for _ in range(50):
        cfg.one(cmd(), 3, True)
    for i in range(5):
        cfg.connect(i)
    cfg.one(cmd(), 5, True)


def wait(cfg, index, n, start_term):               # config.go:535-566
    to = 1
    for _ in range(30):
        nd, _ = cfg.n_committed(index)
        if nd >= n:
            break
        cfg.advance(to)
        to = min(to * 2, 100)
        if start_term > -1:
            for p in range(cfg.P):
                t, _ = cfg.get_state(p)
                if t > start_term:
                    return -1
    nd, cmd = cfg.n_committed(index)
    if nd < n:
        raise HarnessFailure(f"only {nd} decided for index {index}; wanted {n}")
    return cmd


def persist1_2c(mk, seed=8):                         # test_test.go:685-729
    servers = 3
    cfg = Cluster(mk, servers, seed=seed)
    cfg.one(11, servers, True)
    for i in range(servers):                         # crash and re-start all
        cfg.start1(i)
    for i in range(servers):
        cfg.disconnect(i)
        cfg.connect(i)
    cfg.one(12, servers, True)
    leader1 = cfg.check_one_leader()
    cfg.disconnect(leader1)
    cfg.start1(leader1)
    cfg.connect(leader1)
    cfg.one(13, servers, True)
    leader2 = cfg.check_one_leader()
    cfg.disconnect(leader2)
    cfg.one(14, servers - 1, True)
    cfg.start1(leader2)
    cfg.connect(leader2)
    wait(cfg, 4, servers, -1)                        # leader2 joins before i3 is killed
    i3 = (cfg.check_one_leader() + 1) % servers
    cfg.disconnect(i3)
    cfg.one(15, servers - 1, True)
    cfg.start1(i3)
    cfg.connect(i3)
    cfg.one(16, servers, True)


def persist2_2c(mk, seed=9):                         # test_test.go:731-775
    servers = 5
    cfg = Cluster(mk, servers, seed=seed)
    index = 1
    for _ in range(5):
        cfg.one(10 + index, servers, True)
        index += 1
        leader1 = cfg.check_one_leader()
        cfg.disconnect((leader1 + 1) % servers)
        cfg.disconnect((leader1 + 2) % servers)
        cfg.one(10 + index, servers - 2, True)
        index += 1
        for k in (0, 3, 4):
            cfg.disconnect((leader1 + k) % servers)
        cfg.start1((leader1 + 1) % servers)
        cfg.start1((leader1 + 2) % servers)
        cfg.connect((leader1 + 1) % servers)
        cfg.connect((leader1 + 2) % servers)
        cfg.advance(RAFT_ELECTION_TIMEOUT)
        cfg.start1((leader1 + 3) % servers)
        cfg.connect((leader1 + 3) % servers)
        cfg.one(10 + index, servers - 2, True)
        index += 1
        cfg.connect((leader1 + 4) % servers)
        cfg.connect((leader1 + 0) % servers)
    cfg.one(1000, servers, True)


def persist3_2c(mk, seed=10):                        # test_test.go:777-806
    servers = 3
    cfg = Cluster(mk, servers, seed=seed)
    cfg.one(101, 3, True)
    leader = cfg.check_one_leader()
    cfg.disconnect((leader + 2) % servers)
    cfg.one(102, 2, True)
    cfg.crash1((leader + 0) % servers)
    cfg.crash1((leader + 1) % servers)
    cfg.connect((leader + 2) % servers)
    cfg.start1((leader + 0) % servers)
    cfg.connect((leader + 0) % servers)
    cfg.one(103, 2, True)
    cfg.start1((leader + 1) % servers)
    cfg.connect((leader + 1) % servers)
    cfg.one(104, servers, True)


def figure8_2c(mk, seed=11, iters=150):             # test_test.go:817-871 (1000 iterations there)
    servers = 5
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed)
    cfg.one(int(rng.integers(1, 1 << 30)), 1, True)
    nup = servers
    for _ in range(iters):
        leader = -1
        for i in range(servers):
            if cfg.alive[i]:
                _, _, ok = cfg.start(i, int(rng.integers(1, 1 << 30)))
                if ok:
                    leader = i
        if rng.integers(0, 1000) < 100:
            cfg.advance(int(rng.integers(0, RAFT_ELECTION_TIMEOUT // 2)) + 1)
        else:
            cfg.advance(int(rng.integers(0, 13)) // TICK_MS + 1)
        if leader != -1:
            cfg.crash1(leader)
            nup -= 1
        if nup < 3:
            s_ = int(rng.integers(0, servers))
            if not cfg.alive[s_]:
                cfg.start1(s_)
                cfg.connect(s_)
                nup += 1
    for i in range(servers):
        if not cfg.alive[i]:
            cfg.start1(i)
            cfg.connect(i)
    cfg.one(int(rng.integers(1, 1 << 30)), servers, True)


SCENARIOS = {
    "InitialElection2A": initial_election_2a,
    "ReElection2A": re_election_2a,
    "BasicAgree2B": basic_agree_2b,
    "FailAgree2B": fail_agree_2b,
    "FailNoAgree2B": fail_no_agree_2b,
    "Rejoin2B": rejoin_2b,
    "Backup2B": backup_2b,
    "Persist12C": persist1_2c,
    "Persist22C": persist2_2c,
    "Persist32C": persist3_2c,
    "Figure82C": figure8_2c,
}
