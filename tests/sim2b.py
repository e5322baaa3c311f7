"""Deterministic discrete-time counterpart of the reference's Raft test harness
(src/raft/config.go) driving Raft groups through the engine's C ABI — config
#1 of BASELINE.json ("src/raft 3-peer single group via labrpc harness, go test
-run 2B"), and the same scenarios on thousands of groups at once. Test
infrastructure.

`MultiSim` holds G independent Raft groups of P servers in ONE engine (slot
g*P + p is server p of group g) on a shared 10 ms clock. Every group runs its
own scenario of src/raft/test_test.go (a generator: it yields when it waits
for time to pass or needs the engine) with its own seed, network randomness,
partitions, crashes and snapshots; each tick the harness makes one batched
engine call per phase for all groups together — RequestVote deliveries and
tallies, the gather -> HandleAppendEntries -> reply fold rounds (the messages
of many groups' leaders in one call: message sets), InstallSnapshot, the
applier, Snapshot, persistence flushes and restarts — so the batched paths run
on realistic mixed histories. With G = 1 it is the single-group replay.

Mapping to the reference:
  * time advances in 10 ms ticks; heartbeats every 90 ms (raft.go:42-44),
    randomized election timeouts 300-600 ms (raft.go:46-50), seeded per group;
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
    engine marked persist_dirty are saved to the Persister
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
    bytes, SnapshotValid messages (raft.go:168-177, the applier's snapshot
    output) ingested as ingestSnap does (:183-209); a leader whose
    nextIndex[p]-1 is below its dummy sends InstallSnapshot
    (raft_append_entry.go:27-39) carrying its persisted snapshot; start1
    ingests the persisted snapshot before Make (:306-316);
  * RPC counts (labrpc.go:366-383, config.go rpcCount) count the requests a
    connected server received (dropped requests included, as labrpc counts
    them before the drop); RPC bytes (labrpc.go:159,288,292, bytesTotal) add
    the gob-sized request of every such request and every delivered reply —
    an AppendEntries carries its entries' commands (RpcBytes2B).
Commands never enter the engine: the harness keeps each server's commands
index-aligned with its log (the host side of the boundary, include/mraft.h).
"""
from __future__ import annotations

import json
import os
import sys
from dataclasses import dataclass

import numpy as np

from multiraft_amd._abi import (AE_RESULT, F_BECAME_LEADER, F_NEED_MORE, F_SNAPSHOT_INSTALLED,
                                F_STEPPED_DOWN, IS_RESULT, ITEM_NEED_SNAPSHOT, LEADER, RV_ARGS, RV_RESULT)
from multiraft_amd.engine import new_state
from multiraft_amd.persister import Persister, flush_persist, restart

TICK_MS = 10
HEARTBEAT = 9          # ticks
ELECTION = (30, 60)    # ticks
RAFT_ELECTION_TIMEOUT = 100  # ticks = 1 s (test_test.go:22)
SNAPSHOT_INTERVAL = 10       # config.go:215
MAXLOGSIZE = 2000            # test_test.go:1110 (bytes of persisted raft state; our codec's size)

# gob-sized RPC records (labrpc counts len(gob bytes), labrpc.go:159,288,292):
# a struct of small ints is a few tens of bytes on the wire; an Entry adds its
# Index/Term/Id and the command (a string's length, else a varint)
RPC_HEADER_BYTES = 64
RPC_REPLY_BYTES = 32
ENTRY_BYTES = 24


def cmd_bytes(cmd) -> int:
    return len(cmd) if isinstance(cmd, (str, bytes)) else 8


class HarnessFailure(AssertionError):
    pass


class Cluster:
    """One Raft group of P servers inside a MultiSim: the group's own host
    state (config.go's cfg), and the scenario-facing API. Methods that wait
    for time or need the engine are generators (`yield from`)."""

    def __init__(self, sim: "MultiSim", g: int, seed: int, unreliable: bool = False, snap: bool = False):
        P = sim.P
        self.sim, self.g, self.P, self.L = sim, g, P, sim.L
        self.base = g * P
        self.rng = np.random.default_rng(seed)
        self.net = np.random.default_rng(seed + 7919)  # labrpc's randomness
        self.connected = sim.connected[g]             # views into the sim's [G, P] arrays
        self.alive = sim.alive[g]                     # cfg.rafts[i] != nil
        self.elec = sim.elec[g]
        self.hb = sim.hb[g]
        for p in range(P):
            self.elec[p] = self._etimeout()
        self.cmds = [dict() for _ in range(P)]      # host command mirror: index -> cmd
        self.logs = [dict() for _ in range(P)]      # cfg.logs: applied index -> cmd
        self.max_index = 0
        self.rpcs = 0
        self.rpc_count = [0] * P                    # labrpc GetCount(server): requests received
        self.bytes_total = 0                        # labrpc GetTotalBytes
        self.saved_cmds = [dict() for _ in range(P)]  # commands persisted beside the raft state
        self.unreliable = unreliable                # labrpc Reliable(false)
        self.long_reordering = False                # labrpc LongReordering(true)
        self.delayed = []                           # replies in flight: (tick, kind, record)
        self.snap = snap                            # applierSnap (config.go:212-268)
        self.last_applied = [0] * P                 # cfg.lastApplied
        self.snap_bytes = [b""] * P                 # the snapshot each server's Snapshot()/install saves
        self.installs = 0                           # InstallSnapshot handled with an install
        self.count_bytes = False                    # RPC bytes of AppendEntries entries (RPCBytes2B)
        self.done = False

    # ---- helpers ---------------------------------------------------------
    @property
    def now(self):
        return self.sim.now

    def _etimeout(self):
        return self.sim.now + int(self.rng.integers(ELECTION[0], ELECTION[1]))

    def role(self, p):
        return int(self.sim.st["state"][self.base + p])

    def term(self, p):
        return int(self.sim.st["current_term"][self.base + p])

    def _link(self, a, b):
        return self.connected[a] and self.connected[b] and self.alive[a] and self.alive[b]

    def setunreliable(self, on: bool):
        self.unreliable = on

    def setlongreordering(self, on: bool):
        self.long_reordering = on

    def _req_ok(self, a, b, nbytes=RPC_HEADER_BYTES):
        """A request from a to b: connected, received (counted), not dropped."""
        if not self._link(a, b):
            return False
        self.rpc_count[b] += 1
        self.bytes_total += nbytes
        return not (self.unreliable and self.net.integers(0, 1000) < 100)

    def _reply_delay(self):
        """Ticks until the reply arrives; None: dropped (labrpc.go:270-290)."""
        if self.unreliable and self.net.integers(0, 1000) < 100:
            return None
        self.bytes_total += RPC_REPLY_BYTES
        if self.long_reordering and self.net.integers(0, 900) < 600:
            return (200 + int(self.net.integers(0, 1 + int(self.net.integers(0, 2000))))) // TICK_MS
        return int(self.net.integers(0, 3)) if self.unreliable else 0

    def read_snapshot(self, p):
        return self.sim.persister.read_snapshot(self.base + p)

    def log_size(self):
        """config.go LogSize: the largest persisted raft state."""
        return max(self.sim.persister.raft_state_size(self.base + p) for p in range(self.P))

    def crash1(self, p):
        """config.go:112-142: disconnect, kill; the persisted bytes survive."""
        self.disconnect(p)
        self.alive[p] = False

    def start1(self, p):
        """config.go:283-340: crash1, then Make + readPersist from the saved
        state; the server stays disconnected until connect()."""
        yield ("start1", p)

    def connect(self, p):
        self.connected[p] = True

    def disconnect(self, p):
        self.connected[p] = False

    # ---- Raft API mirror --------------------------------------------------
    def start(self, p, cmd, replicate: bool = True):
        """Raft.Start (raft.go:90-104) on server p (+ BroadcastAppend)."""
        if not self.alive[p]:
            return -1, -1, False
        return (yield ("start", p, cmd, replicate))

    def replicate(self, leaders):
        """BroadcastAppend from the given servers now (+ persistence flush)."""
        yield ("replicate", list(leaders))

    def get_state(self, p):
        """GetState (raft.go:237-246)."""
        return self.term(p), self.role(p) == LEADER

    def advance(self, ticks):
        if ticks > 0:
            yield ("wait", int(ticks))

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

    def _apply_slot(self, p, fr, to, si):
        """The applier's messages of server p (raft.go:153-203) as config.go's
        applier / applierSnap consume them; returns the Snapshot(index) the
        service takes, or -1."""
        snap_at = -1
        if si >= 0:                                          # SnapshotValid (raft.go:168-177)
            if not self.snap:
                raise HarnessFailure(f"server {p}: SnapshotValid without snapshots")
            self._ingest_snap(p, self.snap_bytes[p], si)     # CondInstallSnapshot: true
        for i in range(fr, to + 1):
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
                snap_at = i
        return snap_at

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
            yield from self.advance(int(self.rng.integers(45, 56)))
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
                    idx, _, ok = yield from self.start(starts, cmd)
                    if ok:
                        index = idx
                        break
            if index != -1:
                t1 = self.now
                while self.now - t1 < 200:
                    nd, c = self.n_committed(index)
                    if nd > 0 and nd >= expected and c == cmd:
                        return index
                    yield from self.advance(2)
                if not retry:
                    raise HarnessFailure(f"one({cmd}) failed to reach agreement")
            else:
                yield from self.advance(5)
        raise HarnessFailure(f"one({cmd}) failed to reach agreement")


class MultiSim:
    """G Raft groups of P servers (L-entry log capacity) in ONE engine,
    every group running its own scenario; see the module docstring."""

    def __init__(self, make_backend, P: int, L: int, specs, compact_apply: bool = False):
        """specs: [(scenario, seed)] with scenario a `Scenario`, one per group."""
        G = len(specs)
        self.G, self.P, self.L = G, P, L
        self.eng = make_backend(G, P, L, new_state(G, P, L))
        self.compact_apply = compact_apply and hasattr(self.eng, "collect_apply_compact")
        self.now = 0
        self.connected = np.ones((G, P), bool)
        self.alive = np.ones((G, P), bool)
        self.elec = np.zeros((G, P), np.int64)
        self.hb = np.zeros((G, P), np.int64)
        self.persister = Persister(G * P)           # cfg.saved, slot = g*P + p
        self.groups = [Cluster(self, g, seed, sc.unreliable, sc.snap) for g, (sc, seed) in enumerate(specs)]
        self.specs = specs
        self.failures = {}
        self.calls = {}                              # engine call -> (calls, items)
        self._refresh()

    # ---- engine plumbing ---------------------------------------------------
    def _call(self, name, *a, n=0, **kw):
        c = self.calls.setdefault(name, [0, 0])
        c[0] += 1
        c[1] += n
        return getattr(self.eng, name)(*a, **kw)

    def _refresh(self):
        """Host mirror of the replica scalars (roles, terms) after every batch."""
        if hasattr(self.eng, "scalar_state"):
            self.st = self.eng.scalar_state()
        else:
            self.st = self.eng.store_state()

    def _fail(self, g, exc):
        if g not in self.failures:
            self.failures[g] = exc
        grp = self.groups[g]
        grp.done = True
        self.alive[g, :] = False                      # the group stops; the others go on

    def _flush(self):
        """The persist() call sites of the last batch, saved (persister.go);
        SaveStateAndSnapshot marks save the snapshot bytes the server made
        (Snapshot) or received (InstallSnapshot)."""
        P = self.P
        for s in flush_persist(self.eng, self.persister, lambda s: self.groups[s // P].snap_bytes[s % P]):
            g, p = divmod(int(s), P)
            self.groups[g].saved_cmds[p] = dict(self.groups[g].cmds[p])

    # ---- scheduling ----------------------------------------------------------
    def run(self, max_ticks: int = 400000):
        gens = {g: sc.fn(self.groups[g], seed) for g, (sc, seed) in enumerate(self.specs)}
        wake = {g: 0 for g in gens}
        progress = int(os.environ.get("MRAFT_SIM_PROGRESS", "0"))  # print every N ticks (long GPU runs)
        while gens:
            if progress and self.now % progress == 0:
                print(f"[sim] tick {self.now}: {len(gens)} of {self.G} groups running", file=sys.stderr, flush=True)
            ready = [g for g in sorted(gens) if wake[g] <= self.now]
            if ready:
                self._resume(gens, wake, ready)
            if not gens:
                break
            self._step()
            if self.now > max_ticks:
                raise HarnessFailure(f"simulation passed {max_ticks} ticks")
        if self.failures:
            g, exc = min(self.failures.items())
            if self.G == 1:
                raise exc
            names = {}
            for gg in self.failures:
                names.setdefault(self.specs[gg][0].name, []).append(gg)
            raise HarnessFailure(f"{len(self.failures)} of {self.G} groups failed "
                                 f"({ {k: v[:5] for k, v in names.items()} }); first: group {g} "
                                 f"{self.specs[g][0].name}: {exc}")
        return self

    def _resume(self, gens, wake, ready):
        """Runs the ready groups' scenarios until each waits for time; the
        engine requests they make meanwhile are served in batches."""
        to_send = {g: None for g in ready}
        while to_send:
            reqs = {"start": [], "start1": [], "replicate": []}
            for g, val in to_send.items():
                if self.groups[g].done:
                    gens.pop(g).close()
                    continue
                try:
                    r = gens[g].send(val)
                except StopIteration:
                    del gens[g]
                    self.groups[g].done = True
                    self.alive[g, :] = False                  # finished: the group goes quiet
                    continue
                except AssertionError as e:                   # the scenario's own checks
                    del gens[g]
                    self._fail(g, e)
                    continue
                if r[0] == "wait":
                    wake[g] = self.now + r[1]
                else:
                    reqs[r[0]].append((g,) + tuple(r[1:]))
            to_send = {}
            if reqs["start1"]:
                self._start1(reqs["start1"])
                to_send.update({g: None for g, *_ in reqs["start1"]})
            if reqs["start"]:
                to_send.update(self._start(reqs["start"]))
            if reqs["replicate"]:
                self._replicate({g: ls for g, ls in reqs["replicate"]})
                self._flush()
                to_send.update({g: None for g, _ in reqs["replicate"]})

    # ---- one tick ---------------------------------------------------------
    def _step(self):
        self.now += 1
        P = self.P
        self._deliver_delayed()
        self._refresh()
        role = self.st["state"].reshape(self.G, P)
        cands = {}
        for g, p in np.argwhere(self.alive & (self.now >= self.elec)):
            self.elec[g, p] = self.groups[g]._etimeout()
            if role[g, p] != LEADER:
                cands.setdefault(int(g), []).append(int(p))
        if cands:
            self._election(cands)
        self._refresh()
        role = self.st["state"].reshape(self.G, P)
        leaders = {}
        for g, p in np.argwhere(self.alive & (role == LEADER) & (self.now >= self.hb)):
            leaders.setdefault(int(g), []).append(int(p))
        if leaders:
            self._replicate(leaders)
        self._flush()
        self._apply()

    # ---- Start / restart ----------------------------------------------------
    def _start(self, reqs):
        """Raft.Start for one server of each requesting group (one call), then
        BroadcastAppend(Append) from the ones that lead."""
        P = self.P
        slots = np.array([g * P + p for g, p, *_ in reqs], np.int32)
        idx, term, isl, err = self._call("start", slots, n=len(slots))
        assert not err.any(), err
        out, rep = {}, {}
        for k, (g, p, cmd, replicate) in enumerate(reqs):
            if not isl[k]:
                out[g] = (-1, -1, False)
                continue
            self.groups[g].cmds[p][int(idx[k])] = cmd
            out[g] = (int(idx[k]), int(term[k]), True)
            if replicate:
                rep[g] = [p]
        self._flush()
        self._refresh()
        if rep:
            self._replicate(rep)
            self._flush()
        return out

    def _start1(self, reqs):
        P = self.P
        slots = []
        for g, p in reqs:
            grp = self.groups[g]
            grp.crash1(p)
            grp.last_applied[p] = 0                     # :302
            snapb = self.persister.read_snapshot(g * P + p)
            if grp.snap and snapb:                      # :306-316 ingestSnap before Make
                grp._ingest_snap(p, snapb, -1)
            grp.snap_bytes[p] = snapb
            slots.append(g * P + p)
        self.calls.setdefault("restore", [0, 0])[0] += 1
        err = restart(self.eng, self.persister, slots)
        assert not err.any(), err
        for g, p in reqs:
            grp = self.groups[g]
            grp.cmds[p] = dict(grp.saved_cmds[p])
            grp.alive[p] = True
            grp.elec[p] = grp._etimeout()
            grp.hb[p] = 0
        self._refresh()

    # ---- elections --------------------------------------------------------
    def _election(self, cands):
        """StartElection for every candidate; RequestVote deliveries one round
        per candidate rank (each group's k-th candidate in round k: a voter
        gets at most one request per call); one tally call for all."""
        P = self.P
        order = [(g, c) for g in sorted(cands) for c in cands[g]]
        args, err = self._call("start_election", np.array([g * P + c for g, c in order], np.int32), n=len(order))
        assert not err.any(), err
        arg = {gc: args[i] for i, gc in enumerate(order)}
        results = {gc: [] for gc in order}
        for ci in range(max(len(v) for v in cands.values())):
            items, meta = [], []
            for g in sorted(cands):
                if ci >= len(cands[g]):
                    continue
                c, grp = cands[g][ci], self.groups[g]
                a = arg[(g, c)]
                for v in range(P):
                    if v == c or not grp._req_ok(c, v):
                        continue
                    items.append((g * P + v, a["candidate_id"], a["term"], a["last_log_index"], a["last_log_term"]))
                    meta.append((g, c, v))
                    grp.rpcs += 1
            if not items:
                continue
            rep, rerr = self._call("handle_request_vote", np.array(items, dtype=RV_ARGS), n=len(items))
            assert not rerr.any(), rerr
            for (g, c, v), r in zip(meta, rep):
                grp = self.groups[g]
                if r["vote_granted"]:
                    grp.elec[v] = grp._etimeout()                # raft_election.go:72
                rec = (g * P + c, v, int(arg[(g, c)]["term"]), int(r["term"]), int(r["vote_granted"]))
                d = grp._reply_delay()
                if d is None:
                    continue
                if d > 0:
                    grp.delayed.append((self.now + d, "rv", rec))
                else:
                    results[(g, c)].append(rec)
        items, seg = [], [0]
        for gc in order:
            items += results[gc]
            if results[gc]:
                seg.append(len(items))
        if items:
            self._tally(items, seg)

    def _tally(self, items, seg):
        flags, ferr = self._call("process_vote_replies", np.array(items, dtype=RV_RESULT),
                                 np.array(seg, np.int64), n=len(items))
        assert not ferr.any(), ferr
        new = {}
        for s in sorted({items[i][0] for i in range(len(items)) if flags[i] & F_BECAME_LEADER}):
            g, p = divmod(int(s), self.P)
            new.setdefault(g, []).append(p)
        # (the tally's step-down resets no timer in the reference)
        if new:
            self._refresh()
            self._replicate(new)                                  # BroadcastAppend(HeartBeat)

    def _deliver_delayed(self):
        """Replies whose (reordered) arrival time has come, in arrival order
        per group (each group's k-th due reply in the k-th batch)."""
        dues = {}
        for g, grp in enumerate(self.groups):
            if not grp.delayed:
                continue
            due = [d for d in grp.delayed if d[0] <= self.now]
            if due:
                grp.delayed = [d for d in grp.delayed if d[0] > self.now]
                due.sort(key=lambda d: d[0])
                dues[g] = due
        if not dues:
            return
        for k in range(max(len(v) for v in dues.values())):
            rv, ae, is_ = [], [], []
            for g, due in dues.items():
                if k >= len(due) or self.groups[g].done:
                    continue
                _, kind, rec = due[k]
                if not self.alive[g, rec[0] % self.P]:
                    continue                                      # the sender was killed meanwhile
                (rv if kind == "rv" else ae if kind == "ae" else is_).append(rec)
            if rv:
                self._tally(rv, list(range(len(rv) + 1)))
            if ae:
                self._fold(ae)
            if is_:
                self._fold_is(is_)
        self._flush()
        self._apply()

    # ---- replication -------------------------------------------------------
    def _replicate(self, leaders, max_rounds=16):
        """BroadcastAppend rounds for {group: [leaders]}: per round one
        gather, the InstallSnapshots, one HandleAppendEntries call per
        leader rank (each group's j-th leader in call j: a follower receives
        at most one message per call) and one reply fold; a group goes on
        while one of its followers still needs entries."""
        P = self.P
        active = {g: list(ls) for g, ls in leaders.items()}
        for _ in range(max_rounds):
            if not active:
                return
            self._refresh()
            role = self.st["state"]
            slots, peers, owner = [], [], []
            for g in sorted(active):
                grp = self.groups[g]
                for ld in active[g]:
                    if role[g * P + ld] != LEADER or not grp.alive[ld]:
                        continue
                    grp.hb[ld] = self.now + HEARTBEAT
                    for p in range(P):
                        if p != ld:
                            slots.append(g * P + ld)
                            peers.append(p)
                            owner.append(g)
            if not slots:
                return
            args, gerr = self._call("gather_append_args", np.array(slots, np.int32), np.array(peers, np.int32),
                                    n=len(slots))
            snaps = [i for i in range(len(slots)) if gerr[i] == ITEM_NEED_SNAPSHOT]
            deliver = []
            for i in range(len(slots)):
                if gerr[i] != 0:
                    continue
                grp = self.groups[owner[i]]
                nb = RPC_HEADER_BYTES
                if grp.count_bytes:
                    ld, pv = slots[i] % P, int(args[i]["prev_log_index"])
                    nb += sum(ENTRY_BYTES + cmd_bytes(grp.cmds[ld].get(x))
                              for x in range(pv + 1, pv + 1 + int(args[i]["n_entries"])))
                if grp._req_ok(slots[i] % P, peers[i], nb):
                    deliver.append(i)
            more = self._install_snapshots([(owner[i], slots[i], peers[i]) for i in snaps])
            by = {}
            for i in deliver:
                by.setdefault(owner[i], {}).setdefault(slots[i], []).append(i)
            per = {g: list(d.values()) for g, d in by.items()}
            results = []
            for j in range(max((len(v) for v in per.values()), default=0)):
                idx = [i for g in sorted(per) if j < len(per[g]) for i in per[g][j]]
                a = args[idx]
                rep, herr = self._call("handle_append_entries", a, None, n=len(idx))
                assert not herr.any(), herr
                for k, i in enumerate(idx):
                    g, f, ld = owner[i], peers[i], slots[i] % P
                    grp, r = self.groups[g], rep[k]
                    grp.rpcs += 1
                    if not (r["term"] > a[k]["term"]):                   # not the stale path:
                        grp.elec[f] = grp._etimeout()                    # :121 timer reset
                    if r["success"]:
                        prev, n = int(a[k]["prev_log_index"]), int(a[k]["n_entries"])
                        src, dst = grp.cmds[ld], grp.cmds[f]
                        for x in range(prev + 1, prev + n + 1):          # host command mirror
                            dst[x] = src.get(x)
                    rec = (slots[i], f, int(a[k]["term"]), int(a[k]["prev_log_index"]), int(a[k]["n_entries"]),
                           int(r["term"]), int(r["success"]), int(r["conflict_index"]))
                    d = grp._reply_delay()
                    if d is None:
                        continue
                    if d > 0:
                        grp.delayed.append((self.now + d, "ae", rec))
                    else:
                        results.append(rec)
            if results:
                more |= self._fold(results)
            self._apply()
            active = {g: ls for g, ls in active.items() if g in more}

    def _segments(self, recs):
        recs = sorted(recs, key=lambda t: (t[0], t[1]))
        seg, cur = [0], None
        for i, t in enumerate(recs):
            if cur is not None and t[0] != cur:
                seg.append(i)
            cur = t[0]
        seg.append(len(recs))
        return recs, seg

    def _fold(self, results):
        """processAppendEntriesReply for delivered replies, one segment per
        leader; returns the groups where some leader still needs to send
        (:84-86)."""
        results, seg = self._segments(results)
        flags, ferr = self._call("process_append_replies", np.array(results, dtype=AE_RESULT),
                                 np.array(seg, np.int64), n=len(results))
        assert not ferr.any(), ferr
        more = set()
        for i, t in enumerate(results):
            g, ld = divmod(t[0], self.P)
            if flags[i] & F_STEPPED_DOWN:
                grp = self.groups[g]
                grp.elec[ld] = grp._etimeout()                   # :71 timer reset
            if flags[i] & F_NEED_MORE:
                more.add(g)
        return more

    def _install_snapshots(self, items):
        """The snapshot branch of appendOneRound (raft_append_entry.go:27-39):
        InstallSnapshot with the leader's persisted snapshot, the follower's
        HandleInstallSnapshot (raft_snapshot.go:15-54) and the leader's
        processInstallSnapshotReply (:56-69). Returns the groups that sent
        one."""
        if not items:
            return set()
        P = self.P
        args, gerr = self._call("gather_install_snapshot_args", np.array([s for _, s, _ in items], np.int32),
                                np.array([p for _, _, p in items], np.int32), n=len(items))
        sel = []
        for k, (g, s, p) in enumerate(items):
            if gerr[k] == 0 and args["slot"][k] >= 0:
                grp = self.groups[g]
                nb = RPC_HEADER_BYTES + len(grp.snap_bytes[s % P])
                if grp._req_ok(s % P, p, nb):
                    sel.append(k)
        if not sel:
            return set()
        a = args[sel]
        rep, fl, herr = self._call("handle_install_snapshot", a, n=len(sel))
        assert not herr.any(), herr
        recs, sent = [], set()
        for j, k in enumerate(sel):
            g, s, f = items[k]
            grp, ld = self.groups[g], s % P
            sent.add(g)
            grp.rpcs += 1
            if rep["term"][j] <= a["term"][j]:
                grp.elec[f] = grp._etimeout()                    # raft_snapshot.go:29 timer reset
            if fl[j] & F_SNAPSHOT_INSTALLED:
                grp.snap_bytes[f] = grp.snap_bytes[ld]           # args.Snapshot, saved at :47
                grp.installs += 1
            rec = (s, f, int(a["term"][j]), int(a["last_included_index"][j]), int(rep["term"][j]))
            d = grp._reply_delay()
            if d is None:
                continue
            if d > 0:
                grp.delayed.append((self.now + d, "is", rec))
            else:
                recs.append(rec)
        self._flush()
        if recs:
            self._fold_is(recs)
        return sent

    def _fold_is(self, recs):
        recs, seg = self._segments(recs)
        fl, err = self._call("process_install_snapshot_replies", np.array(recs, dtype=IS_RESULT),
                             np.array(seg, np.int64), n=len(recs))
        assert not err.any(), err
        for i, t in enumerate(recs):
            if fl[i] & F_STEPPED_DOWN:
                g, ld = divmod(t[0], self.P)
                grp = self.groups[g]
                grp.elec[ld] = grp._etimeout()

    # ---- applier -------------------------------------------------------------
    def _apply(self):
        P = self.P
        if self.compact_apply:
            sl, si, _, fr, to, n = self._call("collect_apply_compact", snapshots=True, n=1)
            assert n == len(sl)
        else:
            fr, to, si, _ = self._call("collect_apply", snapshots=True, n=1)
            sl = np.nonzero((to >= fr) | (si >= 0))[0]
            fr, to, si = fr[sl], to[sl], si[sl]
        snaps = {}
        for k, s in enumerate(sl):
            g, p = divmod(int(s), P)
            grp = self.groups[g]
            if not grp.alive[p] or grp.done:
                continue
            try:
                i = grp._apply_slot(p, int(fr[k]), int(to[k]), int(si[k]))
            except HarnessFailure as e:
                self._fail(g, e)
                continue
            if i >= 0:
                snaps[int(s)] = i
        if snaps:
            # Snapshot(i) for every qualifying index in apply order; the last one
            # per server decides the state (Snapshot trims monotonically and the
            # engine takes one item per replica per call)
            err = self._call("snapshot", np.array(list(snaps), np.int32), np.array(list(snaps.values()), np.int32),
                             n=len(snaps))
            assert not err.any(), err
            self._flush()


@dataclass
class Scenario:
    name: str
    fn: object
    P: int
    L: int = 512
    unreliable: bool = False
    snap: bool = False


def run_scenario(mk, name, seed):
    """One scenario on one group (G = 1): the single-group replay."""
    sc = SCENARIOS[name]
    return MultiSim(mk, sc.P, sc.L, [(sc, seed)]).run()


def run_many(mk, names, n_groups, seed0=1000, P=None, L=None, compact_apply=False):
    """n_groups independent groups in ONE engine, group g running scenario
    names[g % len(names)] with seed seed0 + g (all scenarios must share P)."""
    scs = [SCENARIOS[n] for n in names]
    P = P or scs[0].P
    assert all(s.P == P for s in scs), "one engine: every scenario needs the same server count"
    L = L or max(s.L for s in scs)
    specs = [(scs[g % len(scs)], seed0 + g) for g in range(n_groups)]
    return MultiSim(mk, P, L, specs, compact_apply=compact_apply).run()


# ---------------------------------------------------------------------------
# Scenarios: the assertions of src/raft/test_test.go (generators over a Cluster)
# ---------------------------------------------------------------------------

def initial_election_2a(cfg, seed):                  # test_test.go:24-53
    yield from cfg.check_one_leader()
    yield from cfg.advance(5)
    t1 = cfg.check_terms()
    assert t1 >= 1, "term is 0 after election"
    yield from cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    cfg.check_terms()  # the reference only warns if the term changed (:45-47)
    yield from cfg.check_one_leader()


def re_election_2a(cfg, seed):                       # test_test.go:55-93
    l1 = yield from cfg.check_one_leader()
    cfg.disconnect(l1)
    yield from cfg.check_one_leader()
    cfg.connect(l1)
    l2 = yield from cfg.check_one_leader()
    cfg.disconnect(l2)
    cfg.disconnect((l2 + 1) % 3)
    yield from cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    assert not any(cfg.connected[p] and cfg.role(p) == LEADER for p in range(3)), "leader without majority"
    cfg.connect((l2 + 1) % 3)
    yield from cfg.check_one_leader()
    cfg.connect(l2)
    yield from cfg.check_one_leader()


def basic_agree_2b(cfg, seed):                       # test_test.go:128-153
    for index in range(1, 4):
        nd, _ = cfg.n_committed(index)
        assert nd == 0, "some have committed before Start()"
        x = yield from cfg.one(index * 100, 3, False)
        assert x == index, f"got index {x} but expected {index}"


def randstring(rng, n):                              # test_test.go randstring: base64 of n random bytes, cut to n
    import base64
    return base64.urlsafe_b64encode(rng.bytes(n)).decode()[:n]


def rpc_bytes_2b(cfg, seed):                         # test_test.go:155-187
    servers = 3
    rng = np.random.default_rng(seed)
    cfg.count_bytes = True
    yield from cfg.one(99, servers, False)
    bytes0 = cfg.bytes_total
    iters, sent = 10, 0
    for index in range(2, iters + 2):
        cmd = randstring(rng, 5000)
        xindex = yield from cfg.one(cmd, servers, False)
        assert xindex == index, f"got index {xindex} but expected {index}"
        sent += len(cmd)
    got = cfg.bytes_total - bytes0
    expected = servers * sent
    assert got <= expected + 50000, f"too many RPC bytes; got {got}, expected {expected}"
    cfg.rpc_bytes_result = (got, expected)


def fail_agree_2b(cfg, seed):                        # test_test.go:279-311
    yield from cfg.one(101, 3, False)
    leader = yield from cfg.check_one_leader()
    cfg.disconnect((leader + 1) % 3)
    yield from cfg.one(102, 2, False)
    yield from cfg.one(103, 2, False)
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT)
    yield from cfg.one(104, 2, False)
    yield from cfg.one(105, 2, False)
    cfg.connect((leader + 1) % 3)
    yield from cfg.one(106, 3, True)
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT)
    yield from cfg.one(107, 3, True)


def fail_no_agree_2b(cfg, seed):                     # test_test.go:313-362
    yield from cfg.one(10, 5, False)
    leader = yield from cfg.check_one_leader()
    for k in (1, 2, 3):
        cfg.disconnect((leader + k) % 5)
    index, _, ok = yield from cfg.start(leader, 20)
    assert ok, "leader rejected Start()"
    assert index == 2, f"expected index 2, got {index}"
    yield from cfg.advance(2 * RAFT_ELECTION_TIMEOUT)
    n, _ = cfg.n_committed(index)
    assert n == 0, f"{n} committed but no majority"
    for k in (1, 2, 3):
        cfg.connect((leader + k) % 5)
    leader2 = yield from cfg.check_one_leader()
    index2, _, ok2 = yield from cfg.start(leader2, 30)
    assert ok2, "leader2 rejected Start()"
    assert 2 <= index2 <= 3, f"unexpected index {index2}"
    yield from cfg.one(1000, 5, True)


def rejoin_2b(cfg, seed):                            # test_test.go:465-501
    yield from cfg.one(101, 3, True)
    leader1 = yield from cfg.check_one_leader()
    cfg.disconnect(leader1)
    yield from cfg.start(leader1, 102)
    yield from cfg.start(leader1, 103)
    yield from cfg.start(leader1, 104)
    yield from cfg.one(103, 2, True)
    leader2 = yield from cfg.check_one_leader()
    cfg.disconnect(leader2)
    cfg.connect(leader1)
    yield from cfg.one(104, 2, True)
    cfg.connect(leader2)
    yield from cfg.one(105, 3, True)


def backup_2b(cfg, seed):                            # test_test.go:503-573
    rng = np.random.default_rng(seed)
    cmd = lambda: int(rng.integers(1, 1 << 30))  # noqa: E731
    yield from cfg.one(cmd(), 5, True)
    leader1 = yield from cfg.check_one_leader()
    for k in (2, 3, 4):
        cfg.disconnect((leader1 + k) % 5)
    for _ in range(50):
        yield from cfg.start(leader1, cmd())
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT // 2)
    cfg.disconnect((leader1 + 0) % 5)
    cfg.disconnect((leader1 + 1) % 5)
    for k in (2, 3, 4):
        cfg.connect((leader1 + k) % 5)
    for _ in range(50):
        yield from cfg.one(cmd(), 3, True)
    leader2 = yield from cfg.check_one_leader()
    other = (leader1 + 2) % 5
    if leader2 == other:
        other = (leader2 + 1) % 5
    cfg.disconnect(other)
    for _ in range(50):
        yield from cfg.start(leader2, cmd())
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT // 2)
    for i in range(5):
        cfg.disconnect(i)
    cfg.connect((leader1 + 0) % 5)
    cfg.connect((leader1 + 1) % 5)
    cfg.connect(other)
    for _ in range(50):
        yield from cfg.one(cmd(), 3, True)
    for i in range(5):
        cfg.connect(i)
    yield from cfg.one(cmd(), 5, True)


def wait(cfg, index, n, start_term):               # config.go:535-566
    to = 1
    for _ in range(30):
        nd, _ = cfg.n_committed(index)
        if nd >= n:
            break
        yield from cfg.advance(to)
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


def persist1_2c(cfg, seed):                          # test_test.go:685-729
    servers = 3
    yield from cfg.one(11, servers, True)
    for i in range(servers):                         # crash and re-start all
        yield from cfg.start1(i)
    for i in range(servers):
        cfg.disconnect(i)
        cfg.connect(i)
    yield from cfg.one(12, servers, True)
    leader1 = yield from cfg.check_one_leader()
    cfg.disconnect(leader1)
    yield from cfg.start1(leader1)
    cfg.connect(leader1)
    yield from cfg.one(13, servers, True)
    leader2 = yield from cfg.check_one_leader()
    cfg.disconnect(leader2)
    yield from cfg.one(14, servers - 1, True)
    yield from cfg.start1(leader2)
    cfg.connect(leader2)
    yield from wait(cfg, 4, servers, -1)             # leader2 joins before i3 is killed
    i3 = ((yield from cfg.check_one_leader()) + 1) % servers
    cfg.disconnect(i3)
    yield from cfg.one(15, servers - 1, True)
    yield from cfg.start1(i3)
    cfg.connect(i3)
    yield from cfg.one(16, servers, True)


def persist2_2c(cfg, seed):                          # test_test.go:731-775
    servers = 5
    index = 1
    for _ in range(5):
        yield from cfg.one(10 + index, servers, True)
        index += 1
        leader1 = yield from cfg.check_one_leader()
        cfg.disconnect((leader1 + 1) % servers)
        cfg.disconnect((leader1 + 2) % servers)
        yield from cfg.one(10 + index, servers - 2, True)
        index += 1
        for k in (0, 3, 4):
            cfg.disconnect((leader1 + k) % servers)
        yield from cfg.start1((leader1 + 1) % servers)
        yield from cfg.start1((leader1 + 2) % servers)
        cfg.connect((leader1 + 1) % servers)
        cfg.connect((leader1 + 2) % servers)
        yield from cfg.advance(RAFT_ELECTION_TIMEOUT)
        yield from cfg.start1((leader1 + 3) % servers)
        cfg.connect((leader1 + 3) % servers)
        yield from cfg.one(10 + index, servers - 2, True)
        index += 1
        cfg.connect((leader1 + 4) % servers)
        cfg.connect((leader1 + 0) % servers)
    yield from cfg.one(1000, servers, True)


def persist3_2c(cfg, seed):                          # test_test.go:777-806
    servers = 3
    yield from cfg.one(101, 3, True)
    leader = yield from cfg.check_one_leader()
    cfg.disconnect((leader + 2) % servers)
    yield from cfg.one(102, 2, True)
    cfg.crash1((leader + 0) % servers)
    cfg.crash1((leader + 1) % servers)
    cfg.connect((leader + 2) % servers)
    yield from cfg.start1((leader + 0) % servers)
    cfg.connect((leader + 0) % servers)
    yield from cfg.one(103, 2, True)
    yield from cfg.start1((leader + 1) % servers)
    cfg.connect((leader + 1) % servers)
    yield from cfg.one(104, servers, True)


def figure8_2c(cfg, seed, iters=150):               # test_test.go:817-871 (1000 iterations there)
    servers = 5
    rng = np.random.default_rng(seed)
    yield from cfg.one(int(rng.integers(1, 1 << 30)), 1, True)
    nup = servers
    for _ in range(iters):
        leader = -1
        for i in range(servers):
            if cfg.alive[i]:
                _, _, ok = yield from cfg.start(i, int(rng.integers(1, 1 << 30)))
                if ok:
                    leader = i
        if rng.integers(0, 1000) < 100:
            yield from cfg.advance(int(rng.integers(0, RAFT_ELECTION_TIMEOUT // 2)) + 1)
        else:
            yield from cfg.advance(int(rng.integers(0, 13)) // TICK_MS + 1)
        if leader != -1:
            cfg.crash1(leader)
            nup -= 1
        if nup < 3:
            s_ = int(rng.integers(0, servers))
            if not cfg.alive[s_]:
                yield from cfg.start1(s_)
                cfg.connect(s_)
                nup += 1
    for i in range(servers):
        if not cfg.alive[i]:
            yield from cfg.start1(i)
            cfg.connect(i)
    yield from cfg.one(int(rng.integers(1, 1 << 30)), servers, True)


def many_elections_2a(cfg, seed, iters=10):         # test_test.go:95-126
    servers = 7
    rng = np.random.default_rng(seed)
    yield from cfg.check_one_leader()
    for _ in range(1, iters):
        i1, i2, i3 = (int(rng.integers(0, servers)) for _ in range(3))
        cfg.disconnect(i1)
        cfg.disconnect(i2)
        cfg.disconnect(i3)
        yield from cfg.check_one_leader()  # the current leader is alive, or the other four elect one
        cfg.connect(i1)
        cfg.connect(i2)
        cfg.connect(i3)
    yield from cfg.check_one_leader()


def concurrent_starts_2b(cfg, seed):                # test_test.go:364-463
    servers = 3
    for attempt in range(5):
        if attempt > 0:
            yield from cfg.advance(300)                  # time.Sleep(3 s)
        leader = yield from cfg.check_one_leader()
        _, term, ok = yield from cfg.start(leader, 1)
        if not ok:
            continue
        idx = []
        for i in range(5):                               # the 5 concurrent Start()s, one batch
            ix, term1, ok1 = yield from cfg.start(leader, 100 + i, replicate=False)
            if term1 == term and ok1:
                idx.append(ix)
        yield from cfg.replicate([leader])
        if any(cfg.get_state(j)[0] != term for j in range(servers)):
            continue
        cmds, failed = [], False
        for index in idx:
            c = yield from wait(cfg, index, servers, term)
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


def count_2b(cfg, seed):                             # test_test.go:575-680
    servers = 3
    rng = np.random.default_rng(seed)

    def rpcs():
        return sum(cfg.rpc_count)
    yield from cfg.check_one_leader()
    total1 = rpcs()
    assert 1 <= total1 <= 30, f"too many or few RPCs ({total1}) to elect initial leader"
    total2, success = 0, False
    for attempt in range(5):
        if attempt > 0:
            yield from cfg.advance(300)
        leader = yield from cfg.check_one_leader()
        total1 = rpcs()
        iters = 10
        starti, term, ok = yield from cfg.start(leader, 1)
        if not ok:
            continue
        cmds, retry = [], False
        for i in range(1, iters + 2):
            x = int(rng.integers(0, 1 << 31))
            cmds.append(x)
            index1, term1, ok1 = yield from cfg.start(leader, x)
            if term1 != term or not ok1:
                retry = True
                break
            assert starti + i == index1, "Start() failed"
        if retry:
            continue
        for i in range(1, iters + 1):
            c = yield from wait(cfg, starti + i, servers, term)
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
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT)
    total3 = rpcs()
    assert total3 - total2 <= 3 * 20, f"too many RPCs ({total3 - total2}) for 1 second of idleness"


def unreliable_agree_2c(cfg, seed, iters=50):       # test_test.go:873-900
    servers = 5
    for it in range(1, iters):
        for j in range(4):                               # the 4 concurrent clients, one after another
            yield from cfg.one(100 * it + j, 1, True)
        yield from cfg.one(it, 1, True)
    cfg.setunreliable(False)
    yield from cfg.one(100, servers, True)


def figure8_unreliable_2c(cfg, seed, iters=400):    # test_test.go:902-955 (1000 iterations there)
    servers = 5
    rng = np.random.default_rng(seed)
    yield from cfg.one(int(rng.integers(0, 10000)), 1, True)
    nup = servers
    for it in range(iters):
        if it == iters // 5:
            cfg.setlongreordering(True)
        leader = -1
        for i in range(servers):
            _, _, ok = yield from cfg.start(i, int(rng.integers(0, 10000)))
            if ok and cfg.connected[i]:
                leader = i
        if rng.integers(0, 1000) < 100:
            yield from cfg.advance(int(rng.integers(0, RAFT_ELECTION_TIMEOUT // 2)) + 1)
        else:
            yield from cfg.advance(int(rng.integers(0, 13)) // TICK_MS + 1)
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
    yield from cfg.one(int(rng.integers(0, 10000)), servers, True)


def _churn(cfg, seed):                               # test_test.go:957-1098 internalChurn
    servers = 5
    rng = np.random.default_rng(seed)
    # three clients Start() on every server without end: logs grow well past
    # the default capacity (the engine rejects an append beyond L)
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
                    ix, _, ok1 = yield from cfg.start(i, x)
                    if ok1:
                        ok, index = True, ix
            if ok:
                c["wait"] = (x, index, cfg.now + 38)
            else:
                c["next"] = cfg.now + (79 + me * 17) // TICK_MS

    def advance(t):
        for _ in range(t):
            yield from cfg.advance(1)
            yield from run_clients()
    for _ in range(20):
        if rng.integers(0, 1000) < 200:
            cfg.disconnect(int(rng.integers(0, servers)))
        if rng.integers(0, 1000) < 500:
            i = int(rng.integers(0, servers))
            if not cfg.alive[i]:
                yield from cfg.start1(i)
            cfg.connect(i)
        if rng.integers(0, 1000) < 200:
            i = int(rng.integers(0, servers))
            if cfg.alive[i]:
                cfg.crash1(i)
        yield from advance(RAFT_ELECTION_TIMEOUT * 7 // 10)
    yield from advance(RAFT_ELECTION_TIMEOUT)
    cfg.setunreliable(False)
    for i in range(servers):
        if not cfg.alive[i]:
            yield from cfg.start1(i)
        cfg.connect(i)
    for c in clients:                                    # stop: outstanding waits end
        c["wait"] = None
    yield from cfg.advance(RAFT_ELECTION_TIMEOUT)
    last_index = yield from cfg.one(int(rng.integers(1, 1 << 40)), servers, True)
    really = []
    for index in range(1, last_index + 1):
        really.append((yield from wait(cfg, index, servers, -1)))
    for v in values:
        assert v in really, "didn't find a value"
    assert values, "no client value was ever committed"


def reliable_churn_2c(cfg, seed):                    # test_test.go:1100-1102
    yield from _churn(cfg, seed)


def unreliable_churn_2c(cfg, seed):                  # test_test.go:1104-1106
    yield from _churn(cfg, seed)


def snapcommon(cfg, seed, disconnect, reliable, crash, iters=30):  # test_test.go:1112-1174
    servers = 3
    rng = np.random.default_rng(seed)
    rnd = lambda: int(rng.integers(0, 1 << 40))  # noqa: E731
    yield from cfg.one(rnd(), servers, True)
    leader1 = yield from cfg.check_one_leader()
    for i in range(iters):
        victim, sender = (leader1 + 1) % servers, leader1
        if i % 3 == 1:
            sender, victim = (leader1 + 1) % servers, leader1
        if disconnect:
            cfg.disconnect(victim)
            yield from cfg.one(rnd(), servers - 1, True)
        if crash:
            cfg.crash1(victim)
            yield from cfg.one(rnd(), servers - 1, True)
        nn = SNAPSHOT_INTERVAL // 2 + int(rng.integers(0, SNAPSHOT_INTERVAL))
        for _ in range(nn):                              # perhaps enough to get a snapshot
            yield from cfg.start(sender, rnd())
        if not disconnect and not crash:
            yield from cfg.one(rnd(), servers, True)     # all caught up: no InstallSnapshot needed
        else:
            yield from cfg.one(rnd(), servers - 1, True)
        if cfg.log_size() >= MAXLOGSIZE:
            raise HarnessFailure("Log size too large")
        if disconnect:                                   # a follower that may need a snapshot
            cfg.connect(victim)
            yield from cfg.one(rnd(), servers, True)
            leader1 = yield from cfg.check_one_leader()
        if crash:
            yield from cfg.start1(victim)
            cfg.connect(victim)
            yield from cfg.one(rnd(), servers, True)
            leader1 = yield from cfg.check_one_leader()


def snapshot_basic_2d(cfg, seed):                    # test_test.go:1176-1178
    yield from snapcommon(cfg, seed, False, True, False)


def snapshot_install_2d(cfg, seed):                  # :1180-1182
    yield from snapcommon(cfg, seed, True, True, False)
    assert cfg.installs > 0, "no InstallSnapshot was exercised"


def snapshot_install_unreliable_2d(cfg, seed):       # :1184-1187
    yield from snapcommon(cfg, seed, True, False, False)


def snapshot_install_crash_2d(cfg, seed):            # :1189-1191
    yield from snapcommon(cfg, seed, False, True, True)


def snapshot_install_uncrash_2d(cfg, seed):          # :1193-1195
    yield from snapcommon(cfg, seed, False, False, True)


def snapshot_all_crash_2d(cfg, seed, iters=5):       # test_test.go:1202-1238
    servers = 3
    rng = np.random.default_rng(seed)
    rnd = lambda: int(rng.integers(0, 1 << 40))  # noqa: E731
    yield from cfg.one(rnd(), servers, True)
    for _ in range(iters):
        nn = SNAPSHOT_INTERVAL // 2 + int(rng.integers(0, SNAPSHOT_INTERVAL))
        for _ in range(nn):
            yield from cfg.one(rnd(), servers, True)
        index1 = yield from cfg.one(rnd(), servers, True)
        for i in range(servers):                         # crash all
            cfg.crash1(i)
        for i in range(servers):                         # revive all, from snapshot + log tail
            yield from cfg.start1(i)
            cfg.connect(i)
        index2 = yield from cfg.one(rnd(), servers, True)
        assert index2 >= index1 + 1, f"index decreased from {index1} to {index2}"
    assert any(cfg.read_snapshot(p) for p in range(servers)), "no snapshot was persisted"


_S = Scenario
SCENARIOS = {s.name: s for s in [
    _S("InitialElection2A", initial_election_2a, 3),
    _S("ReElection2A", re_election_2a, 3),
    _S("BasicAgree2B", basic_agree_2b, 3),
    _S("RPCBytes2B", rpc_bytes_2b, 3),
    _S("FailAgree2B", fail_agree_2b, 3),
    _S("FailNoAgree2B", fail_no_agree_2b, 5),
    _S("Rejoin2B", rejoin_2b, 3),
    _S("Backup2B", backup_2b, 5),
    _S("Persist12C", persist1_2c, 3),
    _S("Persist22C", persist2_2c, 5),
    _S("Persist32C", persist3_2c, 3),
    _S("Figure82C", figure8_2c, 5),
    _S("ManyElections2A", many_elections_2a, 7),
    _S("ConcurrentStarts2B", concurrent_starts_2b, 3),
    _S("Count2B", count_2b, 3),
    _S("UnreliableAgree2C", unreliable_agree_2c, 5, unreliable=True),
    _S("Figure8Unreliable2C", figure8_unreliable_2c, 5, unreliable=True),
    _S("ReliableChurn2C", reliable_churn_2c, 5, L=8192),
    _S("UnreliableChurn2C", unreliable_churn_2c, 5, L=8192, unreliable=True),
    _S("SnapshotBasic2D", snapshot_basic_2d, 3, snap=True),
    _S("SnapshotInstall2D", snapshot_install_2d, 3, snap=True),
    _S("SnapshotInstallUnreliable2D", snapshot_install_unreliable_2d, 3, unreliable=True, snap=True),
    _S("SnapshotInstallCrash2D", snapshot_install_crash_2d, 3, snap=True),
    _S("SnapshotInstallUnCrash2D", snapshot_install_uncrash_2d, 3, unreliable=True, snap=True),
    _S("SnapshotAllCrash2D", snapshot_all_crash_2d, 3, snap=True),
]}
