"""Second, independent CPU restatement of the reference's Raft decision logic.

TEST INFRASTRUCTURE ONLY — imported by tests/ (and tests/golden/make_golden.py)
as a checker; never by the product package.

Unlike the C oracle (oracle/mraft_oracle.c), which works on the device's
struct-of-arrays layout, this restatement keeps the reference's own object
shapes: a `Raft` object per replica with a `logs` list of `Entry(Index, Term)`
(src/raft/raft.go:16-40, src/raft/raft_log.go:3-12, src/raft/raft_rpc.go:39-44)
and message objects mirroring raft_rpc.go:55-82. Agreement between the two
restatements on randomized states is one of the pins of the oracle (the
reference itself cannot run here: no Go toolchain). Pure-Python loops: use
only on small cases.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

LEADER, CANDIDATE, FOLLOWER = 1, 2, 3  # raft_rpc.go:8-12

# item errors / flags (include/mraft.h)
ITEM_OK, PREV_BEYOND_LAST, BELOW_DUMMY, LOG_FULL, NEED_SNAPSHOT, DUP_SLOT, BAD_SLOT, BAD_STATE = range(8)
F_NEED_MORE, F_COMMITTED, F_STEPPED_DOWN, F_BECAME_LEADER, F_APPLIED = 1, 2, 4, 8, 16
G_ACTIVE, G_COMMITTED, G_STEPPED_DOWN, G_NEED_SNAPSHOT, G_ERROR, G_FOLLOWER_COMMIT, G_LOG_FULL = 1, 2, 4, 8, 16, 32, 64
G_ELECTED, G_SNAPSHOT_INSTALLED, G_FOLLOWER_PANIC = 128, 256, 512
F_SNAPSHOT_INSTALLED = 32


class Panic(Exception):
    """A Go panic (raft_log.go:56-58, raft_append_entry.go:41-43)."""


@dataclass
class Entry:  # raft_rpc.go:39-44 (Command/Id never influence decisions)
    Index: int
    Term: int


@dataclass
class AppendEntriesArgs:  # raft_rpc.go:55-62
    Term: int
    LeaderId: int
    Entries: List[Entry]
    PrevLogIndex: int
    PrevLogTerm: int
    LeaderCommit: int


@dataclass
class AppendEntriesReply:  # raft_rpc.go:64-69
    Conflict: bool = False
    ConflictIndex: int = 0
    Term: int = 0
    Success: bool = False


@dataclass
class RequestVoteArgs:  # raft_rpc.go:71-76
    CandidateId: int
    Term: int
    LastLogIndex: int
    LastLogTerm: int


@dataclass
class InstallSnapshotArgs:  # raft_rpc.go:84-90 (Snapshot bytes omitted)
    Term: int
    LeaderId: int
    LastIncludedIndex: int
    LastIncludedTerm: int


@dataclass
class InstallSnapshotReply:  # raft_rpc.go:92-95
    Term: int = 0
    Success: bool = False


@dataclass
class RequestVoteReply:  # raft_rpc.go:78-82
    Term: int = 0
    VoteGranted: bool = False


class RaftLog:  # raft_log.go:3-104
    def __init__(self, logs: List[Entry]):
        self.logs = logs

    def dummyIndex(self):
        return self.logs[0].Index

    def dummyTerm(self):
        return self.logs[0].Term

    def convertIndex(self, index):
        if index < self.dummyIndex():
            raise Panic("current index is smaller than dummy Index")
        return index - self.dummyIndex()

    def getEntry(self, index):
        return self.logs[self.convertIndex(index)]

    def lastIndex(self):
        return self.logs[-1].Index

    def lastTerm(self):
        return self.logs[-1].Term

    def lastEntry(self):
        return self.logs[-1]

    def append(self, *ents):
        self.logs.extend(ents)
        return self.lastIndex()

    def trunc(self, high):
        self.logs = self.logs[: self.convertIndex(high)]
        return self.lastIndex()

    def sliceFrom(self, low):
        return self.logs[self.convertIndex(low):]

    def len(self):
        return len(self.logs)

    def setLogs(self, newlogs):  # raft_log.go:18-21 (copy)
        self.logs = [Entry(e.Index, e.Term) for e in newlogs]

    def matchLog(self, Term, Index):
        return Index <= self.lastIndex() and Term == self.getEntry(Index).Term

    def isLogUpToDate(self, requestLastTerm, requestLastIndex):
        my = self.lastEntry()
        return requestLastTerm > my.Term or (my.Term == requestLastTerm and requestLastIndex >= my.Index)


@dataclass
class Raft:  # raft.go:16-40 (decision-relevant fields)
    me: int
    npeers: int
    currentTerm: int
    votedFor: int
    state: int
    raftLog: RaftLog
    commitIndex: int
    lastApplied: int
    nextIndex: List[int]
    matchIndex: List[int]
    grantedVotes: int = 0
    persisted: int = 0  # persist() (1) / SaveStateAndSnapshot() (1|2) ran since the last collect
    hasSnapshot: bool = False  # raft.go:158, set by HandleInstallSnapshot (raft_snapshot.go:52)

    def persist(self, bits=1):  # raft.go:205-208; SaveStateAndSnapshot persister.go:58-63
        self.persisted |= bits

    # ---- raft_append_entry.go ----
    def gatherArgs(self, peer):  # appendOneRound :20-54 (args part)
        if self.state != LEADER:
            return None, BAD_STATE
        prevLogIndex = self.nextIndex[peer] - 1
        if prevLogIndex < self.raftLog.dummyIndex():
            return None, NEED_SNAPSHOT
        if prevLogIndex > self.raftLog.lastIndex():
            return None, PREV_BEYOND_LAST  # panic in Go
        args = AppendEntriesArgs(
            LeaderId=self.me, Term=self.currentTerm, PrevLogIndex=prevLogIndex,
            PrevLogTerm=self.raftLog.getEntry(prevLogIndex).Term,
            Entries=[Entry(e.Index, e.Term) for e in self.raftLog.sliceFrom(prevLogIndex + 1)],
            LeaderCommit=self.commitIndex)
        return args, ITEM_OK

    def processAppendEntriesReply(self, peer, args, reply):  # :66-88
        flags = 0
        if reply.Term > self.currentTerm:
            self.currentTerm = reply.Term
            self.votedFor = -1
            self.state = FOLLOWER
            self.persist()  # :72
            flags |= F_STEPPED_DOWN
        elif (reply.Term == self.currentTerm and self.state == LEADER and
              args.Term == self.currentTerm and args.PrevLogIndex == self.nextIndex[peer] - 1):
            flags |= F_APPLIED
            if reply.Success:
                self.matchIndex[peer] = len(args.Entries) + args.PrevLogIndex
                self.nextIndex[peer] = self.matchIndex[peer] + 1
                if self.advanceCommitIndexForLeader():
                    flags |= F_COMMITTED
            else:
                self.nextIndex[peer] = reply.ConflictIndex
            if self.nextIndex[peer] < self.raftLog.lastIndex() + 1:
                flags |= F_NEED_MORE
        return flags

    def advanceCommitIndexForLeader(self):  # :89-105
        i = self.raftLog.lastIndex()
        while i > self.commitIndex:
            num = 0
            for j in range(self.npeers):
                if j != self.me and self.matchIndex[j] >= i:
                    num += 1
            if num + 1 > self.npeers // 2 and self.raftLog.getEntry(i).Term == self.currentTerm:
                self.commitIndex = i
                return True
            i -= 1
        return False

    def HandleAppendEntries(self, args, reply):  # :108-162
        self.persist()  # defer rf.persist(), :111
        if args.Term < self.currentTerm:
            reply.Term, reply.Success = self.currentTerm, False
            return
        if args.Term > self.currentTerm:
            self.currentTerm, self.votedFor = args.Term, -1
        self.state = FOLLOWER
        if args.PrevLogIndex < self.raftLog.dummyIndex():
            reply.Term, reply.Success = 0, False
            reply.ConflictIndex = self.raftLog.dummyIndex() + 1
            return
        if not self.raftLog.matchLog(args.PrevLogTerm, args.PrevLogIndex):
            reply.Term, reply.Success = self.currentTerm, False
            lastIndex = self.raftLog.lastIndex()
            if args.PrevLogIndex > lastIndex:
                reply.ConflictIndex = lastIndex + 1
            else:
                dummyIndex = self.raftLog.dummyIndex()
                abandondRound = self.raftLog.getEntry(args.PrevLogIndex).Term
                index = args.PrevLogIndex
                while index > dummyIndex + 1 and self.raftLog.getEntry(index).Term == abandondRound:
                    index -= 1
                reply.ConflictIndex = index
            return
        for index, entry in enumerate(args.Entries):
            if (self.raftLog.convertIndex(entry.Index) >= self.raftLog.len() or
                    self.raftLog.getEntry(entry.Index).Term != entry.Term):
                self.raftLog.trunc(entry.Index)
                self.raftLog.append(*[Entry(e.Index, e.Term) for e in args.Entries[index:]])
                break
        follower_commit = False
        if args.LeaderCommit > self.commitIndex:
            self.commitIndex = min(args.LeaderCommit, self.raftLog.lastIndex())
            follower_commit = True
        reply.Term, reply.Success = self.currentTerm, True
        return follower_commit

    # ---- raft.go ----
    def Start(self):  # raft.go:90-104 (the command stays with the caller)
        if self.state != LEADER:
            return -1, -1, 0
        e = Entry(self.raftLog.lastIndex() + 1, self.currentTerm)
        self.raftLog.append(e)
        self.persist()  # :101
        return e.Index, e.Term, 1

    # ---- raft_snapshot.go ----
    def Snapshot(self, index):  # :3-13
        if index <= self.raftLog.dummyIndex():
            return ITEM_OK
        if index > self.raftLog.lastIndex():
            return PREV_BEYOND_LAST  # sliceFrom panics
        self.raftLog.setLogs(self.raftLog.sliceFrom(index))
        self.persist(3)  # SaveStateAndSnapshot, :12
        return ITEM_OK

    def gatherInstallSnapshot(self):  # raft_append_entry.go:27-34
        return InstallSnapshotArgs(Term=self.currentTerm, LeaderId=self.me,
                                   LastIncludedIndex=self.raftLog.dummyIndex(),
                                   LastIncludedTerm=self.raftLog.dummyTerm())

    def HandleInstallSnapshot(self, args, reply):  # :15-54
        try:
            if args.Term < self.currentTerm:
                return False
            if args.Term > self.currentTerm:
                self.currentTerm, self.votedFor = args.Term, -1
                self.persist()  # :26
            self.state = FOLLOWER
            if args.LastIncludedIndex <= self.commitIndex:
                return False
            if args.LastIncludedIndex > self.raftLog.lastIndex():
                self.raftLog.setLogs([Entry(0, 0)])
            else:
                self.raftLog.setLogs(self.raftLog.sliceFrom(args.LastIncludedIndex))
            self.commitIndex = args.LastIncludedIndex
            self.lastApplied = args.LastIncludedIndex
            self.raftLog.logs[0].Index = args.LastIncludedIndex
            self.raftLog.logs[0].Term = args.LastIncludedTerm
            self.persist(3)  # SaveStateAndSnapshot, :47
            self.hasSnapshot = True  # :52
            return True
        finally:
            reply.Term = self.currentTerm

    def processInstallSnapshotReply(self, peer, args, reply):  # :56-69
        if reply.Term > self.currentTerm:
            self.currentTerm = reply.Term
            self.votedFor = -1
            self.state = FOLLOWER
            self.persist()  # :64
            return F_STEPPED_DOWN
        if self.state == LEADER and args.Term == self.currentTerm:
            self.matchIndex[peer] = args.LastIncludedIndex
            self.nextIndex[peer] = args.LastIncludedIndex + 1
            return F_APPLIED
        return 0

    # ---- raft_election.go ----
    def StartElection(self):  # :4-15
        self.state = CANDIDATE
        self.currentTerm += 1
        lastLog = self.raftLog.lastEntry()
        args = RequestVoteArgs(Term=self.currentTerm, CandidateId=self.me,
                               LastLogIndex=lastLog.Index, LastLogTerm=lastLog.Term)
        self.votedFor = self.me
        self.persist()  # :15
        self.grantedVotes = 1
        return args

    def tally(self, args, reply):  # closure :22-47
        flags = 0
        if self.currentTerm == args.Term and self.state == CANDIDATE:
            if reply.VoteGranted:
                self.grantedVotes += 1
                if self.grantedVotes > self.npeers // 2:
                    self.state = LEADER
                    for i in range(self.npeers):
                        self.matchIndex[i] = 0
                        self.nextIndex[i] = self.raftLog.lastIndex() + 1
                    flags |= F_BECAME_LEADER
            elif reply.Term > self.currentTerm:
                self.state = FOLLOWER
                self.currentTerm, self.votedFor = reply.Term, -1
                self.persist()  # :45
                flags |= F_STEPPED_DOWN
        return flags

    def HandleRequestVote(self, args, reply):  # :54-77
        self.persist()  # defer rf.persist(), :57
        if args.Term < self.currentTerm:
            reply.Term, reply.VoteGranted = self.currentTerm, False
            return
        if args.Term > self.currentTerm:
            self.state = FOLLOWER
            self.currentTerm, self.votedFor = args.Term, -1
        reply.Term = self.currentTerm
        if (self.votedFor == -1 or self.votedFor == args.CandidateId) and \
                self.raftLog.isLogUpToDate(args.LastLogTerm, args.LastLogIndex):
            self.votedFor = args.CandidateId
            reply.VoteGranted = True
            return
        reply.VoteGranted = False


# ---------------------------------------------------------------------------
# SoA <-> objects
# ---------------------------------------------------------------------------

STATE_KEYS = ("current_term", "voted_for", "state", "commit_index", "last_applied",
              "dummy_index", "last_index", "granted_votes", "log_term", "match_index", "next_index", "persist_dirty", "log_head", "has_snapshot")


def from_soa(st: dict, G: int, P: int, L: int) -> List[Raft]:
    rafts = []
    for s in range(G * P):
        d = int(st["dummy_index"][s]); last = int(st["last_index"][s])
        row = st["log_term"][s * L:(s + 1) * L]
        h = int(st["log_head"][s]) if "log_head" in st else 0   # the engine's ring (include/mraft.h)
        logs = [Entry(d + k, int(row[(h + k) % L])) for k in range(last - d + 1)]
        rafts.append(Raft(me=s % P, npeers=P, currentTerm=int(st["current_term"][s]),
                          votedFor=int(st["voted_for"][s]), state=int(st["state"][s]),
                          raftLog=RaftLog(logs), commitIndex=int(st["commit_index"][s]),
                          lastApplied=int(st["last_applied"][s]),
                          nextIndex=[int(x) for x in st["next_index"][s * P:(s + 1) * P]],
                          matchIndex=[int(x) for x in st["match_index"][s * P:(s + 1) * P]],
                          grantedVotes=int(st["granted_votes"][s]),
                          persisted=int(st["persist_dirty"][s]) if "persist_dirty" in st else 0,
                          hasSnapshot=bool(st["has_snapshot"][s]) if "has_snapshot" in st else False))
    return rafts


def to_soa(rafts: List[Raft], st: dict, G: int, P: int, L: int) -> dict:
    """Write objects back into a copy of st (log slots beyond lastIndex keep
    their previous contents, like the device arrays). The object model has no
    ring: each log is written from the replica's existing log_head, so the
    result equals the engine's logically (tests compare logical logs)."""
    out = {k: np.array(v, copy=True) for k, v in st.items() if k != "terms_sorted"}  # engine bookkeeping
    for s, rf in enumerate(rafts):
        out["current_term"][s] = rf.currentTerm
        out["voted_for"][s] = rf.votedFor
        out["state"][s] = rf.state
        out["commit_index"][s] = rf.commitIndex
        out["last_applied"][s] = rf.lastApplied
        out["dummy_index"][s] = rf.raftLog.dummyIndex()
        out["last_index"][s] = rf.raftLog.lastIndex()
        out["granted_votes"][s] = rf.grantedVotes
        if "persist_dirty" not in out:
            out["persist_dirty"] = np.zeros(len(rafts), dtype=np.int32)
        out["persist_dirty"][s] = rf.persisted
        if "has_snapshot" not in out:
            out["has_snapshot"] = np.zeros(len(rafts), dtype=np.int32)
        out["has_snapshot"][s] = int(rf.hasSnapshot)
        if len(rf.raftLog.logs) > L:
            raise ValueError("log exceeds capacity")
        h = int(out["log_head"][s]) if "log_head" in out else 0
        for k, e in enumerate(rf.raftLog.logs):
            out["log_term"][s * L + (h + k) % L] = e.Term
        out["match_index"][s * P:(s + 1) * P] = rf.matchIndex
        out["next_index"][s * P:(s + 1) * P] = rf.nextIndex
    return out


# ---------------------------------------------------------------------------
# Fused tick (same composition as mraft_replicate_tick)
# ---------------------------------------------------------------------------

def replicate_tick(st: dict, G: int, P: int, L: int, leader_peer) -> tuple:
    rafts = from_soa(st, G, P, L)
    gflags = np.zeros(G, dtype=np.int32)
    for g in range(G):
        lp = int(leader_peer[g])
        if lp < 0:
            continue
        if lp >= P:
            gflags[g] = G_ERROR
            continue
        ld = rafts[g * P + lp]
        if ld.state != LEADER:
            continue
        if ld.commitIndex < ld.raftLog.dummyIndex():
            gflags[g] = G_ERROR
            continue
        flags = 0
        ok, snap = {}, {}
        for p in range(P):
            if p == lp:
                continue
            args, err = ld.gatherArgs(p)
            if err == NEED_SNAPSHOT:
                flags |= G_NEED_SNAPSHOT
                snap[p] = ld.gatherInstallSnapshot()
            elif err == PREV_BEYOND_LAST:
                flags |= G_ERROR
            else:
                ok[p] = args
        if flags & G_ERROR:
            gflags[g] = G_ERROR | (flags & G_NEED_SNAPSHOT)
            continue
        flags |= G_ACTIVE
        replies, isreplies = {}, {}
        for p in range(P):
            if p in snap:
                rep = InstallSnapshotReply()
                if _is_would_panic(rafts[g * P + p], snap[p]):
                    flags |= G_FOLLOWER_PANIC
                    continue
                if rafts[g * P + p].HandleInstallSnapshot(snap[p], rep):
                    flags |= G_SNAPSHOT_INSTALLED
                isreplies[p] = rep
                continue
            if p not in ok:
                continue
            args = ok[p]
            fr = rafts[g * P + p]
            if _would_overflow(fr, args, L):
                flags |= G_LOG_FULL
                continue
            reply = AppendEntriesReply()
            fc = fr.HandleAppendEntries(args, reply)
            if fc:
                flags |= G_FOLLOWER_COMMIT
            replies[p] = reply
        c0 = ld.commitIndex
        for p in range(P):
            if p in isreplies:
                fl = ld.processInstallSnapshotReply(p, snap[p], isreplies[p])
            elif p in replies:
                fl = ld.processAppendEntriesReply(p, ok[p], replies[p])
            else:
                continue
            if fl & F_STEPPED_DOWN:
                flags |= G_STEPPED_DOWN
        if ld.commitIndex != c0:
            flags |= G_COMMITTED
        gflags[g] = flags
    return to_soa(rafts, st, G, P, L), gflags


def _is_would_panic(fr: Raft, a: InstallSnapshotArgs) -> bool:
    """HandleInstallSnapshot's sliceFrom below the follower's dummy (Go panic)."""
    lg = fr.raftLog
    return (a.Term >= fr.currentTerm and a.LastIncludedIndex > fr.commitIndex and
            a.LastIncludedIndex <= lg.lastIndex() and a.LastIncludedIndex < lg.dummyIndex())


def _would_overflow(fr: Raft, args: AppendEntriesArgs, L: int) -> bool:
    """Engine capacity rule (include/mraft.h MRAFT_ITEM_LOG_FULL)."""
    lg = fr.raftLog
    if args.Term < fr.currentTerm or args.PrevLogIndex < lg.dummyIndex():
        return False
    if not lg.matchLog(args.PrevLogTerm, args.PrevLogIndex):
        return False
    for e in args.Entries:
        if lg.convertIndex(e.Index) >= lg.len() or lg.getEntry(e.Index).Term != e.Term:
            return args.PrevLogIndex + len(args.Entries) - lg.dummyIndex() > L - 1
    return False


# ---------------------------------------------------------------------------
# Shard controller (src/shardctrler/common.go:53-132), for the router tests
# ---------------------------------------------------------------------------

def realloc_gid(shards, gids, nshards=10):
    """Config.ReAllocGID restated on Python lists (g2s ordered by sorted gid,
    as GetGIDWith{Minimum,Maximum}Shards iterate)."""
    shards = list(shards)
    if not gids:
        return [0] * nshards
    g2s = {g: [] for g in sorted(gids)}
    for s, g in enumerate(shards):
        if g != 0 and g in g2s:
            g2s[g].append(s)

    def gmin():
        idx, mn = -1, nshards + 1
        for g in sorted(g2s):
            if g != 0 and len(g2s[g]) < mn:
                idx, mn = g, len(g2s[g])
        return idx

    def gmax():
        idx, mx = -1, -1
        for g in sorted(g2s):
            if len(g2s[g]) > mx:
                idx, mx = g, len(g2s[g])
        return idx

    for i in range(nshards):
        if shards[i] not in g2s:
            g = gmin()
            shards[i] = g
            g2s[g].append(i)
    while True:
        src, tgt = gmax(), gmin()
        if src != 0 and len(g2s[src]) - len(g2s[tgt]) <= 1:
            break
        g2s[tgt].append(g2s[src].pop(0))
    out = [0] * nshards
    for g, ss in g2s.items():
        for s in ss:
            out[s] = g
    return out
