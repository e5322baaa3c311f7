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
    whose state changed without a persist mark would lose that change here;
  * unreliable networks (labrpc.go:221-312): with `unreliable`, 10 % of the
    requests and 10 % of the replies are dropped and replies take 0-2 ticks;
    with `long_reordering`, 2/3 of the replies arrive 200-2,200 ms late, after
    later ones (non-FIFO: the reply gates of raft_append_entry.go:73-74 and
    raft_election.go:24 decide what a late reply may still change);
  * snapshots (2D): with `snap`, the applier is config.go's applierSnap
    (:212-268): strictly in-order apply, Snapshot(index) every
    SnapShotInterval = 10 entries with the applied commands as the snapshot
    bytes, SnapshotValid messages (raft.go:168-177, mraft_collect_apply's
    snapshot output) ingested as ingestSnap does (:183-209); a leader whose
    nextIndex[p]-1 is below its dummy sends InstallSnapshot
    (raft_append_entry.go:27-39) carrying its persisted snapshot; start1
    ingests the persisted snapshot before Make (:306-316);
  * RPC counts (labrpc.go:366-383, config.go rpcCount) count the requests a
    connected server received (dropped requests included, as labrpc counts
    them before the drop).
Commands never enter the engine: the harness keeps each server's commands
index-aligned with its log (the host side of the boundary, include/mraft.h).
"""
from __future__ import annotations

import json

import numpy as np

from multiraft_amd._abi import (AE_RESULT, F_BECAME_LEADER, F_NEED_MORE, F_SNAPSHOT_INSTALLED,
                                F_STEPPED_DOWN, FOLLOWER, IS_ARGS, IS_RESULT, ITEM_NEED_SNAPSHOT, LEADER,
                                RV_ARGS, RV_RESULT)
from multiraft_amd.engine import new_state
from multiraft_amd.persister import Persister, flush_persist, restart

TICK_MS = 10
HEARTBEAT = 9          # ticks
ELECTION = (30, 60)    # ticks
RAFT_ELECTION_TIMEOUT = 100  # ticks = 1 s (test_test.go:22)
SNAPSHOT_INTERVAL = 10       # config.go:215
MAXLOGSIZE = 2000            # test_test.go:1110 (bytes of persisted raft state; our codec's size)


class HarnessFailure(AssertionError):
    pass


class Cluster:
    """One Raft group of P servers (G = 1) over an engine-like backend."""

    def __init__(self, make_backend, P: int, L: int = 512, seed: int = 1, unreliable: bool = False,
                 snap: bool = False):
        self.P, self.L = P, L
        st = new_state(1, P, L)
        self.eng = make_backend(1, P, L, st)
        self.rng = np.random.default_rng(seed)
        self.net = np.random.default_rng(seed + 7919)  # labrpc's randomness
        self.now = 0
        self.connected = [True] * P
        self.elec = [self._etimeout() for _ in range(P)]
        self.hb = [0] * P
        self.cmds = [dict() for _ in range(P)]      # host command mirror: index -> cmd
        self.logs = [dict() for _ in range(P)]      # cfg.logs: applied index -> cmd
        self.max_index = 0
        self.rpcs = 0
        self.rpc_count = [0] * P                    # labrpc GetCount(server): requests received
        self.alive = [True] * P                     # cfg.rafts[i] != nil
        self.persister = Persister(P)               # cfg.saved
        self.saved_cmds = [dict() for _ in range(P)]  # commands persisted beside the raft state
        self.unreliable = unreliable                # labrpc Reliable(false)
        self.long_reordering = False                # labrpc LongReordering(true)
        self.delayed = []                           # replies in flight: (tick, kind, record)
        self.snap = snap                            # applierSnap (config.go:212-268)
        self.last_applied = [0] * P                 # cfg.lastApplied
        self.snap_bytes = [b""] * P                 # the snapshot each server's Snapshot()/install saves
        self.installs = 0                           # InstallSnapshot handled with an install
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
        """The persist() call sites of the last batch, saved (persister.go);
        SaveStateAndSnapshot marks save the snapshot bytes the server made
        (Snapshot) or received (InstallSnapshot)."""
        for p in flush_persist(self.eng, self.persister, lambda s: self.snap_bytes[s]):
            self.saved_cmds[int(p)] = dict(self.cmds[int(p)])

    def setunreliable(self, on: bool):
        self.unreliable = on

    def setlongreordering(self, on: bool):
        self.long_reordering = on

    def _req_ok(self, a, b):
        """A request from a to b: connected, received (counted), not dropped."""
        if not self._link(a, b):
            return False
        self.rpc_count[b] += 1
        return not (self.unreliable and self.net.integers(0, 1000) < 100)

    def _reply_delay(self):
        """Ticks until the reply arrives; None: dropped (labrpc.go:270-290)."""
        if self.unreliable and self.net.integers(0, 1000) < 100:
            return None
        if self.long_reordering and self.net.integers(0, 900) < 600:
            return (200 + int(self.net.integers(0, 1 + int(self.net.integers(0, 2000))))) // TICK_MS
        return int(self.net.integers(0, 3)) if self.unreliable else 0

    def log_size(self):
        """config.go LogSize: the largest persisted raft state."""
        return max(self.persister.raft_state_size(p) for p in range(self.P))

    def crash1(self, p):
        """config.go:112-142: disconnect, kill; the persisted bytes survive."""
        self.disconnect(p)
        self.alive[p] = False

    def start1(self, p):
        """config.go:283-340: crash1, then Make + readPersist from the saved
        state; the server stays disconnected until connect()."""
        self.crash1(p)
        self.last_applied[p] = 0                    # :302
        snapb = self.persister.read_snapshot(p)
        if self.snap and snapb:                     # :306-316 ingestSnap before Make
            self._ingest_snap(p, snapb, -1)
        self.snap_bytes[p] = snapb
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
    def start(self, p, cmd, replicate: bool = True):
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
        if replicate:
            self._replicate([p])  # BroadcastAppend(Append)
            self._flush()
        return int(idx[0]), int(term[0]), True

    def get_state(self, p):
        """GetState (raft.go:237-246)."""
        return self.term(p), self.role(p) == LEADER

    # ---- one tick ---------------------------------------------------------
    def step(self):
        self.now += 1
        self._deliver_delayed()
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
                if v == c or not self._req_ok(c, v):
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
                rec = (c, v, int(args[ci]["term"]), int(r["term"]), int(r["vote_granted"]))
                d = self._reply_delay()
                if d is None:
                    continue
                if d > 0:
                    self.delayed.append((self.now + d, "rv", rec))
                else:
                    results[c].append(rec)
        items, seg = [], [0]
        for c in cands:
            items += results[c]
            if results[c]:
                seg.append(len(items))
        if not items:
            return
        self._tally(items, seg)

    def _tally(self, items, seg):
        flags, ferr = self.eng.process_vote_replies(np.array(items, dtype=RV_RESULT),
                                                    np.array(seg, np.int64))
        assert not ferr.any(), ferr
        new_leaders = sorted({items[i][0] for i in range(len(items)) if flags[i] & F_BECAME_LEADER})
        # (the tally's step-down resets no timer in the reference)
        if new_leaders:
            self._refresh()
            self._replicate(new_leaders)                      # BroadcastAppend(HeartBeat)

    def _deliver_delayed(self):
        """Replies whose (reordered) arrival time has come, in arrival order."""
        due = [d for d in self.delayed if d[0] <= self.now]
        if not due:
            return
        self.delayed = [d for d in self.delayed if d[0] > self.now]
        due.sort(key=lambda d: d[0])
        for _, kind, rec in due:
            if not self.alive[rec[0]]:
                continue                                      # the sender was killed meanwhile
            if kind == "rv":
                self._tally([rec], [0, 1])
            elif kind == "ae":
                self._fold([rec])
            else:
                self._fold_is([rec])
        self._flush()
        self._apply()

    # ---- replication -------------------------------------------------------
    def _replicate(self, leaders, max_rounds=16):
        for _ in range(max_rounds):
            self._refresh()
            slots, peers = [], []
            for ld in leaders:
                if self.role(ld) != LEADER or not self.alive[ld]:
                    continue
                self.hb[ld] = self.now + HEARTBEAT
                for p in range(self.P):
                    if p != ld:
                        slots.append(ld)
                        peers.append(p)
            if not slots:
                return
            args, gerr = self.eng.gather_append_args(np.array(slots, np.int32), np.array(peers, np.int32))
            snaps = [i for i in range(len(slots)) if gerr[i] == ITEM_NEED_SNAPSHOT]
            deliver = [i for i in range(len(slots)) if gerr[i] == 0 and self._req_ok(slots[i], peers[i])]
            more = self._install_snapshots([slots[i] for i in snaps], [peers[i] for i in snaps])
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
                    rec = (ld, f, int(a[j]["term"]), int(a[j]["prev_log_index"]), int(a[j]["n_entries"]),
                           int(r["term"]), int(r["success"]), int(r["conflict_index"]))
                    d = self._reply_delay()
                    if d is None:
                        continue
                    if d > 0:
                        self.delayed.append((self.now + d, "ae", rec))
                    else:
                        results.append(rec)
            if results:
                more = self._fold(results) or more
            self._apply()
            if not more:
                return

    def _fold(self, results):
        """processAppendEntriesReply for delivered replies, one segment per
        leader; returns whether some leader still needs to send (:84-86)."""
        results = sorted(results, key=lambda t: (t[0], t[1]))
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
        return more

    def _install_snapshots(self, slots, peers):
        """The snapshot branch of appendOneRound (raft_append_entry.go:27-39):
        InstallSnapshot with the leader's persisted snapshot, the follower's
        HandleInstallSnapshot (raft_snapshot.go:15-54) and the leader's
        processInstallSnapshotReply (:56-69)."""
        if not slots:
            return False
        args, gerr = self.eng.gather_install_snapshot_args(np.array(slots, np.int32), np.array(peers, np.int32))
        sel = [i for i in range(len(slots)) if gerr[i] == 0 and args["slot"][i] >= 0
               and self._req_ok(slots[i], peers[i])]
        if not sel:
            return False
        self.rpcs += len(sel)
        a = args[sel]
        rep, fl, herr = self.eng.handle_install_snapshot(a)
        assert not herr.any(), herr
        recs = []
        for j, i in enumerate(sel):
            ld, f = slots[i], peers[i]
            if rep["term"][j] <= a["term"][j]:
                self.elec[f] = self._etimeout()                  # raft_snapshot.go:29 timer reset
            if fl[j] & F_SNAPSHOT_INSTALLED:
                self.snap_bytes[f] = self.snap_bytes[ld]         # args.Snapshot, saved at :47
                self.installs += 1
            rec = (ld, f, int(a["term"][j]), int(a["last_included_index"][j]), int(rep["term"][j]))
            d = self._reply_delay()
            if d is None:
                continue
            if d > 0:
                self.delayed.append((self.now + d, "is", rec))
            else:
                recs.append(rec)
        self._flush()
        if recs:
            self._fold_is(recs)
        return True

    def _fold_is(self, recs):
        recs = sorted(recs, key=lambda t: (t[0], t[1]))
        seg, cur = [0], None
        for i, t in enumerate(recs):
            if cur is not None and t[0] != cur:
                seg.append(i)
            cur = t[0]
        seg.append(len(recs))
        fl, err = self.eng.process_install_snapshot_replies(np.array(recs, dtype=IS_RESULT),
                                                            np.array(seg, np.int64))
        assert not err.any(), err
        for i, t in enumerate(recs):
            if fl[i] & F_STEPPED_DOWN:
                self.elec[t[0]] = self._etimeout()

    # ---- applier + cfg.logs checks (config.go:144-163) --------------------
    def _check_logs(self, p, i, cmd):
        """checkLogs (config.go:144-163): same index => same command."""
        for q in range(self.P):
            if i in self.logs[q] and self.logs[q][i] != cmd:
                raise HarnessFailure(f"commit index={i} server={p} {cmd} != server={q} {self.logs[q][i]}")
        prevok = (i - 1) in self.logs[p]
        self.logs[p][i] = cmd
        self.max_index = max(self.max_index, i)
        return prevok

    def _ingest_snap(self, p, snapb, index):
        """ingestSnap (config.go:183-209)."""
        d = json.loads(snapb.decode())
        if index != -1 and index != d["index"]:
            raise HarnessFailure(f"server {p} snapshot doesn't match m.SnapshotIndex")
        self.logs[p] = {int(k): v for k, v in d["log"].items()}
        self.last_applied[p] = d["index"]

    def _apply(self):
        if not self.snap:
            fr, to = self.eng.collect_apply()
            si = None
        else:
            fr, to, si, _ = self.eng.collect_apply(snapshots=True)
        snaps = []
        for p in range(self.P):
            if not self.alive[p]:
                continue
            if si is not None and si[p] >= 0:                    # SnapshotValid (raft.go:168-177)
                self._ingest_snap(p, self.snap_bytes[p], int(si[p]))   # CondInstallSnapshot: true
            for i in range(int(fr[p]), int(to[p]) + 1):
                cmd = self.cmds[p].get(i)
                if self.snap and i != self.last_applied[p] + 1:  # applierSnap (:232-234)
                    raise HarnessFailure(f"server {p} apply out of order, expected index "
                                         f"{self.last_applied[p] + 1}, got {i}")
                prevok = self._check_logs(p, i, cmd)
                if i > 1 and not prevok:
                    raise HarnessFailure(f"server {p} apply out of order {i}")
                self.last_applied[p] = i
                if self.snap and (i + 1) % SNAPSHOT_INTERVAL == 0:   # :249-262 Snapshot(i, xlog)
                    self.snap_bytes[p] = json.dumps(
                        {"index": i, "log": {j: self.logs[p].get(j) for j in range(i + 1)}}).encode()
                    snaps.append((p, i))
        if snaps:
            # Snapshot(i) for every qualifying index in apply order; the last one
            # per server decides the state (Snapshot trims monotonically and the
            # engine takes one item per replica per call)
            last = {}
            for p, i in snaps:
                last[p] = i
            err = self.eng.snapshot(np.array(list(last), np.int32), np.array(list(last.values()), np.int32))
            assert not err.any(), err
            self._flush()

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


def many_elections_2a(mk, seed=12, iters=10):       # test_test.go:95-126
    servers = 7
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed)
    cfg.check_one_leader()
    for _ in range(1, iters):
        i1, i2, i3 = (int(rng.integers(0, servers)) for _ in range(3))
        cfg.disconnect(i1)
        cfg.disconnect(i2)
        cfg.disconnect(i3)
        cfg.check_one_leader()         # the current leader is alive, or the other four elect one
        cfg.connect(i1)
        cfg.connect(i2)
        cfg.connect(i3)
    cfg.check_one_leader()


def concurrent_starts_2b(mk, seed=13):              # test_test.go:364-463
    servers = 3
    cfg = Cluster(mk, servers, seed=seed)
    for attempt in range(5):
        if attempt > 0:
            cfg.advance(300)                             # time.Sleep(3 s)
        leader = cfg.check_one_leader()
        _, term, ok = cfg.start(leader, 1)
        if not ok:
            continue
        idx = []
        for i in range(5):                               # the 5 concurrent Start()s, one batch
            ix, term1, ok1 = cfg.start(leader, 100 + i, replicate=False)
            if term1 == term and ok1:
                idx.append(ix)
        cfg._replicate([leader])
        cfg._flush()
        if any(cfg.get_state(j)[0] != term for j in range(servers)):
            continue
        cmds, failed = [], False
        for index in idx:
            c = wait(cfg, index, servers, term)
            if c == -1:
                failed = True
                break
            cmds.append(c)
        if failed:
            continue
        for i in range(5):
            assert 100 + i in cmds, f"cmd {100 + i} missing in {cmds}"
        return
    raise HarnessFailure("term changed too often")


def count_2b(mk, seed=14):                           # test_test.go:575-680
    servers = 3
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed)

    def rpcs():
        return sum(cfg.rpc_count)
    cfg.check_one_leader()
    total1 = rpcs()
    assert 1 <= total1 <= 30, f"too many or few RPCs ({total1}) to elect initial leader"
    total2, success = 0, False
    for attempt in range(5):
        if attempt > 0:
            cfg.advance(300)
        leader = cfg.check_one_leader()
        total1 = rpcs()
        iters = 10
        starti, term, ok = cfg.start(leader, 1)
        if not ok:
            continue
        cmds, retry = [], False
        for i in range(1, iters + 2):
            x = int(rng.integers(0, 1 << 31))
            cmds.append(x)
            index1, term1, ok1 = cfg.start(leader, x)
            if term1 != term or not ok1:
                retry = True
                break
            assert starti + i == index1, "Start() failed"
        if retry:
            continue
        for i in range(1, iters + 1):
            c = wait(cfg, starti + i, servers, term)
            if c == -1:
                retry = True
                break
            assert c == cmds[i - 1], f"wrong value {c} committed for index {starti + i}; expected {cmds}"
        if retry:
            continue
        total2 = rpcs()
        if any(cfg.get_state(j)[0] != term for j in range(servers)):
            continue
        assert total2 - total1 <= (iters + 1 + 3) * 3, f"too many RPCs ({total2 - total1}) for {iters} entries"
        success = True
        break
    assert success, "term changed too often"
    cfg.advance(RAFT_ELECTION_TIMEOUT)
    total3 = rpcs()
    assert total3 - total2 <= 3 * 20, f"too many RPCs ({total3 - total2}) for 1 second of idleness"


def unreliable_agree_2c(mk, seed=15, iters=50):      # test_test.go:873-900
    servers = 5
    cfg = Cluster(mk, servers, seed=seed, unreliable=True)
    for it in range(1, iters):
        for j in range(4):                               # the 4 concurrent clients, one after another
            cfg.one(100 * it + j, 1, True)
        cfg.one(it, 1, True)
    cfg.setunreliable(False)
    cfg.one(100, servers, True)


def figure8_unreliable_2c(mk, seed=16, iters=400):   # test_test.go:902-955 (1000 iterations there)
    servers = 5
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed, unreliable=True)
    cfg.one(int(rng.integers(0, 10000)), 1, True)
    nup = servers
    for it in range(iters):
        if it == iters // 5:
            cfg.setlongreordering(True)
        leader = -1
        for i in range(servers):
            _, _, ok = cfg.start(i, int(rng.integers(0, 10000)))
            if ok and cfg.connected[i]:
                leader = i
        if rng.integers(0, 1000) < 100:
            cfg.advance(int(rng.integers(0, RAFT_ELECTION_TIMEOUT // 2)) + 1)
        else:
            cfg.advance(int(rng.integers(0, 13)) // TICK_MS + 1)
        if leader != -1 and rng.integers(0, 1000) < RAFT_ELECTION_TIMEOUT * TICK_MS // 2:
            cfg.disconnect(leader)
            nup -= 1
        if nup < 3:
            s_ = int(rng.integers(0, servers))
            if not cfg.connected[s_]:
                cfg.connect(s_)
                nup += 1
    for i in range(servers):
        if not cfg.connected[i]:
            cfg.connect(i)
    cfg.one(int(rng.integers(0, 10000)), servers, True)


def _churn(mk, seed, unreliable):                    # test_test.go:957-1098 internalChurn
    servers = 5
    rng = np.random.default_rng(seed)
    # three clients Start() on every server without end: logs grow well past
    # the default capacity (the engine rejects an append beyond L)
    cfg = Cluster(mk, servers, L=8192, seed=seed, unreliable=unreliable)
    ncli = 3
    values = []
    # each client: tries Start(x) on every live server, then waits up to 380 ms
    # (10+20+50+100+200) for nCommitted(index); otherwise sleeps 79+me*17 ms
    clients = [{"wait": None, "next": 0} for _ in range(ncli)]

    def run_clients():
        for me, c in enumerate(clients):
            if c["wait"] is not None:
                x, index, deadline = c["wait"]
                nd, cmd = cfg.n_committed(index)
                if nd > 0:
                    if cmd == x:
                        values.append(x)
                    c["wait"] = None
                elif cfg.now >= deadline:
                    c["wait"] = None
                continue
            if cfg.now < c["next"]:
                continue
            x = int(rng.integers(1, 1 << 40))
            index, ok = -1, False
            for i in range(servers):
                if cfg.alive[i]:
                    ix, _, ok1 = cfg.start(i, x)
                    if ok1:
                        ok, index = True, ix
            if ok:
                c["wait"] = (x, index, cfg.now + 38)
            else:
                c["next"] = cfg.now + (79 + me * 17) // TICK_MS

    def advance(t):
        for _ in range(t):
            cfg.step()
            run_clients()
    for _ in range(20):
        if rng.integers(0, 1000) < 200:
            cfg.disconnect(int(rng.integers(0, servers)))
        if rng.integers(0, 1000) < 500:
            i = int(rng.integers(0, servers))
            if not cfg.alive[i]:
                cfg.start1(i)
            cfg.connect(i)
        if rng.integers(0, 1000) < 200:
            i = int(rng.integers(0, servers))
            if cfg.alive[i]:
                cfg.crash1(i)
        advance(RAFT_ELECTION_TIMEOUT * 7 // 10)
    advance(RAFT_ELECTION_TIMEOUT)
    cfg.setunreliable(False)
    for i in range(servers):
        if not cfg.alive[i]:
            cfg.start1(i)
        cfg.connect(i)
    for c in clients:                                    # stop: outstanding waits end
        c["wait"] = None
    cfg.advance(RAFT_ELECTION_TIMEOUT)
    last_index = cfg.one(int(rng.integers(1, 1 << 40)), servers, True)
    really = [wait(cfg, index, servers, -1) for index in range(1, last_index + 1)]
    for v in values:
        assert v in really, "didn't find a value"
    assert values, "no client value was ever committed"


def reliable_churn_2c(mk, seed=17):                  # test_test.go:1100-1102
    _churn(mk, seed, False)


def unreliable_churn_2c(mk, seed=18):                # test_test.go:1104-1106
    _churn(mk, seed, True)


def snapcommon(mk, seed, disconnect, reliable, crash, iters=30):  # test_test.go:1112-1174
    servers = 3
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed, unreliable=not reliable, snap=True)
    rnd = lambda: int(rng.integers(0, 1 << 40))  # noqa: E731
    cfg.one(rnd(), servers, True)
    leader1 = cfg.check_one_leader()
    for i in range(iters):
        victim, sender = (leader1 + 1) % servers, leader1
        if i % 3 == 1:
            sender, victim = (leader1 + 1) % servers, leader1
        if disconnect:
            cfg.disconnect(victim)
            cfg.one(rnd(), servers - 1, True)
        if crash:
            cfg.crash1(victim)
            cfg.one(rnd(), servers - 1, True)
        nn = SNAPSHOT_INTERVAL // 2 + int(rng.integers(0, SNAPSHOT_INTERVAL))
        for _ in range(nn):                              # perhaps enough to get a snapshot
            cfg.start(sender, rnd())
        if not disconnect and not crash:
            cfg.one(rnd(), servers, True)                # all caught up: no InstallSnapshot needed
        else:
            cfg.one(rnd(), servers - 1, True)
        if cfg.log_size() >= MAXLOGSIZE:
            raise HarnessFailure("Log size too large")
        if disconnect:                                   # a follower that may need a snapshot
            cfg.connect(victim)
            cfg.one(rnd(), servers, True)
            leader1 = cfg.check_one_leader()
        if crash:
            cfg.start1(victim)
            cfg.connect(victim)
            cfg.one(rnd(), servers, True)
            leader1 = cfg.check_one_leader()
    return cfg


def snapshot_basic_2d(mk, seed=19):                  # test_test.go:1176-1178
    snapcommon(mk, seed, False, True, False)


def snapshot_install_2d(mk, seed=20):                # :1180-1182
    cfg = snapcommon(mk, seed, True, True, False)
    assert cfg.installs > 0, "no InstallSnapshot was exercised"


def snapshot_install_unreliable_2d(mk, seed=21):     # :1184-1187
    snapcommon(mk, seed, True, False, False)


def snapshot_install_crash_2d(mk, seed=22):          # :1189-1191
    snapcommon(mk, seed, False, True, True)


def snapshot_install_uncrash_2d(mk, seed=23):        # :1193-1195
    snapcommon(mk, seed, False, False, True)


def snapshot_all_crash_2d(mk, seed=24, iters=5):     # test_test.go:1202-1238
    servers = 3
    rng = np.random.default_rng(seed)
    cfg = Cluster(mk, servers, seed=seed, snap=True)
    rnd = lambda: int(rng.integers(0, 1 << 40))  # noqa: E731
    cfg.one(rnd(), servers, True)
    for _ in range(iters):
        nn = SNAPSHOT_INTERVAL // 2 + int(rng.integers(0, SNAPSHOT_INTERVAL))
        for _ in range(nn):
            cfg.one(rnd(), servers, True)
        index1 = cfg.one(rnd(), servers, True)
        for i in range(servers):                         # crash all
            cfg.crash1(i)
        for i in range(servers):                         # revive all, from snapshot + log tail
            cfg.start1(i)
            cfg.connect(i)
        index2 = cfg.one(rnd(), servers, True)
        assert index2 >= index1 + 1, f"index decreased from {index1} to {index2}"
    assert any(cfg.persister.read_snapshot(p) for p in range(servers)), "no snapshot was persisted"


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
    "ManyElections2A": many_elections_2a,
    "ConcurrentStarts2B": concurrent_starts_2b,
    "Count2B": count_2b,
    "UnreliableAgree2C": unreliable_agree_2c,
    "Figure8Unreliable2C": figure8_unreliable_2c,
    "ReliableChurn2C": reliable_churn_2c,
    "UnreliableChurn2C": unreliable_churn_2c,
    "SnapshotBasic2D": snapshot_basic_2d,
    "SnapshotInstall2D": snapshot_install_2d,
    "SnapshotInstallUnreliable2D": snapshot_install_unreliable_2d,
    "SnapshotInstallCrash2D": snapshot_install_crash_2d,
    "SnapshotInstallUnCrash2D": snapshot_install_uncrash_2d,
    "SnapshotAllCrash2D": snapshot_all_crash_2d,
}
