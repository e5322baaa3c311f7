"""Generates tests/golden/kat.json: the known-answer tests K1-K14 of SURVEY.md
§8c, hand-derived from the reference's Go source (cited per case), plus
tests/golden/tick_vectors.npz: seeded replication-tick input/output vectors
produced by the pure-Python restatement (oracle/pyoracle.py).

The reference (Go) cannot run in this image, so the expected values of the
KATs are derived by hand from the cited lines; this script asserts that the
Python restatement reproduces each hand-derived value before writing the
fixture. Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as po  # noqa: E402

LEADER, CANDIDATE, FOLLOWER = 1, 2, 3


def one_group(P, L, slots):
    """slots: {peer: dict(term, voted, state, commit, dummy, terms, match, next)}"""
    st = {k: np.zeros(n, dtype=np.int64) for k, n in {
        "current_term": P, "voted_for": P, "state": P, "commit_index": P, "last_applied": P,
        "dummy_index": P, "last_index": P, "granted_votes": P, "log_term": P * L,
        "match_index": P * P, "next_index": P * P, "persist_dirty": P, "log_head": P, "has_snapshot": P}.items()}
    st["voted_for"][:] = -1
    st["state"][:] = FOLLOWER
    for p in range(P):
        st["log_term"][p * L] = 0
    for p, d in slots.items():
        st["current_term"][p] = d.get("term", 0)
        st["voted_for"][p] = d.get("voted", -1)
        st["state"][p] = d.get("state", FOLLOWER)
        st["commit_index"][p] = d.get("commit", 0)
        st["last_applied"][p] = d.get("commit", 0)
        st["dummy_index"][p] = d.get("dummy", 0)
        terms = d.get("terms", [0])
        st["last_index"][p] = d.get("dummy", 0) + len(terms) - 1
        st["log_term"][p * L:p * L + len(terms)] = terms
        st["match_index"][p * P:(p + 1) * P] = d.get("match", [0] * P)
        st["next_index"][p * P:(p + 1) * P] = d.get("next", [0] * P)
    return {k: v.tolist() for k, v in st.items()}


LT = [0, 1, 1, 2, 2, 3, 3, 4, 4, 4, 4]          # K1-K4 leader log, indices 0..10
FT = [0, 1, 1, 2, 2, 2, 3]                      # K5-K8 follower log, indices 0..6


def commit_kat(name, P, me, match, term, commit, peer, cite, expect):
    """a2 success from `peer` (args rebuilding match[peer]) triggers a1."""
    nxt = [m + 1 for m in match]
    nxt[me] = len(LT)
    m = list(match)
    m[me] = 0
    prev = m[peer] - 1
    nxt[peer] = prev + 1
    st = one_group(P, 16, {me: dict(term=term, voted=me, state=LEADER, commit=commit, terms=LT,
                                    match=m, next=nxt)})
    item = dict(slot=me, peer=peer, args_term=term, args_prev_log_index=prev, args_n_entries=1,
                reply_term=term, reply_success=1, reply_conflict_index=0)
    return dict(name=name, cite=cite, G=1, P=P, L=16, state=st, op="process_append_replies",
                items=[item], expect={"commit_index": {str(me): expect}})


def ae_kat(name, follower, args, cite, expect_reply, expect_state=None, P=3):
    st = one_group(P, 16, {1: follower})
    a = dict(slot=1, term=args["term"], leader_id=0, prev_log_index=args["prev"],
             prev_log_term=args.get("prev_term", 0), leader_commit=args.get("leader_commit", 0),
             n_entries=len(args.get("entries", [])), _pad=0, entries_offset=0)
    return dict(name=name, cite=cite, G=1, P=P, L=16, state=st, op="handle_append_entries",
                args=[a], entry_terms=args.get("entries", []) or [0],
                expect={"reply": expect_reply, "slot1": expect_state or {}})


def rv_kat(name, voter, args, cite, expect_reply, expect_state):
    st = one_group(3, 16, {1: voter})
    a = dict(slot=1, candidate_id=args.get("cand", 2), term=args["term"],
             last_log_index=args["last_idx"], last_log_term=args["last_term"])
    return dict(name=name, cite=cite, G=1, P=3, L=16, state=st, op="handle_request_vote",
                args=[a], expect={"reply": expect_reply, "slot1": expect_state})


def build():
    ae = "src/raft/raft_append_entry.go"
    kats = [
        commit_kat("K1", 5, 0, [0, 7, 5, 3, 9], 4, 2, 1, f"{ae}:89-105", 7),
        commit_kat("K2", 5, 0, [0, 7, 5, 3, 9], 5, 2, 1, f"{ae}:98 (Figure-8 gate)", 2),
        commit_kat("K3", 3, 1, [8, 0, 2], 4, 0, 0, f"{ae}:89-105", 8),
        commit_kat("K4", 4, 0, [0, 9, 7, 3], 4, 2, 1, f"{ae}:98 (P=4 needs 3 of 4)", 7),
        ae_kat("K5", dict(term=3, terms=FT), dict(term=3, prev=5, prev_term=4),
               f"{ae}:136-142 (ConflictIndex is one below the run)",
               dict(term=3, success=0, conflict_index=2)),
        ae_kat("K6", dict(term=3, terms=FT), dict(term=3, prev=9, prev_term=4),
               f"{ae}:131-133", dict(term=3, success=0, conflict_index=7)),
        ae_kat("K7", dict(term=3, terms=[0, 2, 2, 2]), dict(term=3, prev=3, prev_term=5),
               f"{ae}:139 (scan stops at dummy+1)", dict(term=3, success=0, conflict_index=1)),
        ae_kat("K8", dict(term=8, dummy=10, terms=[7, 7, 8]), dict(term=8, prev=8, prev_term=7),
               f"{ae}:123-127 (reply.Term = 0)", dict(term=0, success=0, conflict_index=11)),
        ae_kat("K9", dict(term=2, commit=1, terms=[0, 1, 1, 2, 2, 2]),
               dict(term=3, prev=2, prev_term=1, entries=[2, 2], leader_commit=5),
               f"{ae}:146-160 (no truncation when all match)",
               dict(term=3, success=1, conflict_index=0),
               dict(last_index=5, commit_index=5, current_term=3, voted_for=-1)),
        ae_kat("K10", dict(term=2, commit=1, terms=[0, 1, 1, 2, 2, 2]),
               dict(term=3, prev=2, prev_term=1, entries=[3], leader_commit=5),
               f"{ae}:149-160 (truncate + append, commit vs whole log)",
               dict(term=3, success=1, conflict_index=0),
               dict(last_index=3, commit_index=3, log=[0, 1, 1, 3])),
        rv_kat("K11", dict(term=5, voted=-1, terms=[0] + [4] * 10),
               dict(term=5, last_term=4, last_idx=9), "src/raft/raft_log.go:99-104",
               dict(term=5, vote_granted=0), dict(voted_for=-1)),
        rv_kat("K12", dict(term=5, voted=-1, terms=[0] + [4] * 10),
               dict(term=5, last_term=4, last_idx=10), "src/raft/raft_election.go:69-74",
               dict(term=5, vote_granted=1), dict(voted_for=2)),
        rv_kat("K13", dict(term=5, voted=-1, state=CANDIDATE, terms=[0] + [4] * 10),
               dict(term=6, last_term=3, last_idx=10), "src/raft/raft_election.go:63-67",
               dict(term=6, vote_granted=0), dict(current_term=6, voted_for=-1, state=FOLLOWER)),
    ]
    # K14: tally, P = 7, candidate peer 0: leader at the 3rd granted reply.
    st = one_group(7, 16, {0: dict(term=5, voted=0, state=CANDIDATE, terms=[0, 1, 2])})
    st["granted_votes"][0] = 1
    items = [dict(slot=0, peer=p, args_term=5, reply_term=5, vote_granted=1) for p in (1, 2, 3, 4)]
    kats.append(dict(name="K14", cite="src/raft/raft_election.go:29-38", G=1, P=7, L=16, state=st,
                     op="process_vote_replies", items=items,
                     expect={"flags": [0, 0, 8, 0], "slot0": dict(state=LEADER, granted_votes=4),
                             "next0": [3] * 7, "match0": [0] * 7}))
    # Every handled AppendEntries / RequestVote persists (deferred
    # rf.persist(), raft_append_entry.go:111, raft_election.go:57); a
    # successful reply fold or a granted tally does not.
    for k in kats:
        k["expect"]["persist"] = ({"1": 1} if k["op"] in ("handle_append_entries", "handle_request_vote")
                                  else {str(i): 0 for i in range(k["P"])})
    kats += persist_kats()
    return kats


def persist_kats():
    """P1-P10: the persist() / SaveStateAndSnapshot() call sites (include/mraft.h
    MRAFT_PERSIST_*: 1 = raft state, 2 = snapshot), hand-derived."""
    ae, el, sn, rf = ("src/raft/raft_append_entry.go", "src/raft/raft_election.go",
                      "src/raft/raft_snapshot.go", "src/raft/raft.go")
    FL = [0, 1, 1, 2, 2, 3]  # follower log, indices 0..5
    out = []
    # P1: reply with a higher term -> step down + persist (:67-72)
    st = one_group(3, 16, {0: dict(term=4, voted=0, state=LEADER, commit=1, terms=FL,
                                   match=[0, 1, 1], next=[6, 2, 2])})
    out.append(dict(name="P1", cite=f"{ae}:67-72", G=1, P=3, L=16, state=st, op="process_append_replies",
                    items=[dict(slot=0, peer=1, args_term=4, args_prev_log_index=1, args_n_entries=4,
                                reply_term=6, reply_success=0, reply_conflict_index=0)],
                    expect={"flags": [4], "slot0": dict(current_term=6, voted_for=-1, state=FOLLOWER),
                            "persist": {"0": 1}}))

    def is_kat(name, cite, follower, args, reply_term, persist, extra=None):
        st = one_group(3, 16, {1: follower})
        a = dict(slot=1, term=args["term"], leader_id=0, last_included_index=args["lii"],
                 last_included_term=args["lit"])
        e = {"is_reply": reply_term, "persist": {"1": persist}}
        if extra:
            e["slot1"] = extra
        return dict(name=name, cite=cite, G=1, P=3, L=16, state=st, op="handle_install_snapshot",
                    args=[a], expect=e)
    out.append(is_kat("P2", f"{sn}:20-22 (stale: no persist)", dict(term=5, commit=2, terms=FL),
                      dict(term=4, lii=4, lit=2), 5, 0, dict(current_term=5, dummy_index=0)))
    out.append(is_kat("P3", f"{sn}:31-33 (outdated, same term: no persist)",
                      dict(term=5, commit=4, terms=FL), dict(term=5, lii=3, lit=2), 5, 0,
                      dict(commit_index=4, dummy_index=0)))
    out.append(is_kat("P4", f"{sn}:23-26 (term adopted: persist)", dict(term=5, commit=4, terms=FL),
                      dict(term=7, lii=3, lit=2), 7, 1,
                      dict(current_term=7, voted_for=-1, dummy_index=0, commit_index=4)))
    out.append(is_kat("P5", f"{sn}:38-47 (installed: SaveStateAndSnapshot)",
                      dict(term=5, commit=1, terms=FL), dict(term=5, lii=4, lit=2), 5, 3,
                      dict(dummy_index=4, last_index=5, commit_index=4, last_applied=4, log=[2, 3])))
    # P6: Snapshot below/at dummy is a no-op (:6-9); above it saves state + snapshot (:10-12)
    st = one_group(3, 16, {0: dict(term=3, commit=5, terms=FL), 2: dict(term=3, commit=5, terms=FL, dummy=0)})
    out.append(dict(name="P6", cite=f"{sn}:3-13", G=1, P=3, L=16, state=st, op="snapshot",
                    slots=[0, 2], index=[0, 3],
                    expect={"persist": {"0": 0, "2": 3}, "slot0": dict(dummy_index=0),
                            "slot2": dict(dummy_index=3, log=[2, 2, 3])}))
    # P7: Start on a follower returns early (:93-95); on the leader it persists (:96-101)
    st = one_group(3, 16, {0: dict(term=3, terms=FL), 1: dict(term=3, state=LEADER, voted=1, terms=FL)})
    out.append(dict(name="P7", cite=f"{rf}:90-104", G=1, P=3, L=16, state=st, op="start",
                    slots=[0, 1], expect={"start": [[-1, -1, 0], [6, 3, 1]],
                                          "persist": {"0": 0, "1": 1}, "slot1": dict(last_index=6)}))
    # P8: a denied vote with a higher term -> step down + persist (:42-45)
    st = one_group(3, 16, {0: dict(term=5, voted=0, state=CANDIDATE, terms=[0, 1])})
    st["granted_votes"][0] = 1
    out.append(dict(name="P8", cite=f"{el}:42-45", G=1, P=3, L=16, state=st, op="process_vote_replies",
                    items=[dict(slot=0, peer=1, args_term=5, reply_term=8, vote_granted=0)],
                    expect={"flags": [4], "slot0": dict(state=FOLLOWER, current_term=8, voted_for=-1),
                            "persist": {"0": 1}}))
    # P9: processInstallSnapshotReply with a higher term -> step down + persist (:59-64)
    st = one_group(3, 16, {0: dict(term=4, voted=0, state=LEADER, commit=4, dummy=3, terms=[2, 2, 3],
                                   match=[0, 0, 0], next=[6, 1, 6])})
    out.append(dict(name="P9", cite=f"{sn}:56-69", G=1, P=3, L=16, state=st,
                    op="process_install_snapshot_replies",
                    items=[dict(slot=0, peer=1, args_term=4, args_last_included_index=3, reply_term=9),
                           dict(slot=0, peer=2, args_term=4, args_last_included_index=3, reply_term=4)],
                    expect={"flags": [4, 0], "slot0": dict(current_term=9, state=FOLLOWER),
                            "persist": {"0": 1}}))
    # P10: a stale RequestVote still persists (deferred, :57)
    out.append(rv_kat("P10", dict(term=6, voted=2, terms=[0, 1]), dict(term=4, last_term=9, last_idx=9),
                      f"{el}:57-62", dict(term=6, vote_granted=0), dict(voted_for=2, current_term=6)))
    out[-1]["expect"]["persist"] = {"1": 1}
    return out


def run_py(k):
    """Evaluate a KAT with the pure-Python restatement."""
    G, P, L = k["G"], k["P"], k["L"]
    st = {kk: np.array(v, dtype=np.int32) for kk, v in k["state"].items()}
    rafts = po.from_soa(st, G, P, L)
    out = {}
    if k["op"] == "process_append_replies":
        flags = []
        for it in k["items"]:
            rf = rafts[it["slot"]]
            args = po.AppendEntriesArgs(Term=it["args_term"], LeaderId=rf.me,
                                        Entries=[None] * it["args_n_entries"],
                                        PrevLogIndex=it["args_prev_log_index"], PrevLogTerm=0,
                                        LeaderCommit=0)
            rep = po.AppendEntriesReply(Term=it["reply_term"], Success=bool(it["reply_success"]),
                                        ConflictIndex=it["reply_conflict_index"])
            flags.append(rf.processAppendEntriesReply(it["peer"], args, rep))
        out["flags"] = flags
    elif k["op"] == "handle_append_entries":
        a = k["args"][0]
        rf = rafts[a["slot"]]
        ents = [po.Entry(a["prev_log_index"] + 1 + i, t)
                for i, t in enumerate(k["entry_terms"][:a["n_entries"]])]
        args = po.AppendEntriesArgs(Term=a["term"], LeaderId=a["leader_id"], Entries=ents,
                                    PrevLogIndex=a["prev_log_index"], PrevLogTerm=a["prev_log_term"],
                                    LeaderCommit=a["leader_commit"])
        rep = po.AppendEntriesReply()
        rf.HandleAppendEntries(args, rep)
        out["reply"] = dict(term=rep.Term, success=int(rep.Success), conflict_index=rep.ConflictIndex)
    elif k["op"] == "handle_request_vote":
        a = k["args"][0]
        rf = rafts[a["slot"]]
        rep = po.RequestVoteReply()
        rf.HandleRequestVote(po.RequestVoteArgs(CandidateId=a["candidate_id"], Term=a["term"],
                                                LastLogIndex=a["last_log_index"],
                                                LastLogTerm=a["last_log_term"]), rep)
        out["reply"] = dict(term=rep.Term, vote_granted=int(rep.VoteGranted))
    elif k["op"] == "process_vote_replies":
        flags = []
        for it in k["items"]:
            rf = rafts[it["slot"]]
            flags.append(rf.tally(po.RequestVoteArgs(CandidateId=rf.me, Term=it["args_term"],
                                                     LastLogIndex=0, LastLogTerm=0),
                                  po.RequestVoteReply(Term=it["reply_term"],
                                                      VoteGranted=bool(it["vote_granted"]))))
        out["flags"] = flags
    elif k["op"] == "handle_install_snapshot":
        a = k["args"][0]
        rep = po.InstallSnapshotReply()
        rafts[a["slot"]].HandleInstallSnapshot(po.InstallSnapshotArgs(
            Term=a["term"], LeaderId=a["leader_id"], LastIncludedIndex=a["last_included_index"],
            LastIncludedTerm=a["last_included_term"]), rep)
        out["is_reply"] = rep.Term
    elif k["op"] == "snapshot":
        for s_, x in zip(k["slots"], k["index"]):
            rafts[s_].Snapshot(x)
    elif k["op"] == "start":
        out["start"] = [list(rafts[s_].Start()) for s_ in k["slots"]]
    elif k["op"] == "process_install_snapshot_replies":
        flags = []
        for it in k["items"]:
            rf = rafts[it["slot"]]
            flags.append(rf.processInstallSnapshotReply(
                it["peer"], po.InstallSnapshotArgs(Term=it["args_term"], LeaderId=rf.me,
                                                   LastIncludedIndex=it["args_last_included_index"],
                                                   LastIncludedTerm=0),
                po.InstallSnapshotReply(Term=it["reply_term"])))
        out["flags"] = flags
    out["state"] = po.to_soa(rafts, st, G, P, L)
    return out


def check_kat(k, out):
    """Assert that evaluation output `out` (flags/reply/state) meets k['expect']."""
    e = k["expect"]
    st = out["state"]
    P, L = k["P"], k["L"]
    if "commit_index" in e:
        for s, v in e["commit_index"].items():
            assert st["commit_index"][int(s)] == v, (k["name"], st["commit_index"][int(s)], v)
    if "reply" in e:
        for f, v in e["reply"].items():
            assert out["reply"][f] == v, (k["name"], f, out["reply"][f], v)
    if "is_reply" in e:
        assert out["is_reply"] == e["is_reply"], (k["name"], out["is_reply"], e["is_reply"])
    if "start" in e:
        assert [list(x) for x in out["start"]] == e["start"], (k["name"], out["start"], e["start"])
    for s_, v in e.get("persist", {}).items():
        assert st["persist_dirty"][int(s_)] == v, (k["name"], "persist_dirty", s_,
                                                   st["persist_dirty"][int(s_)], v)
    for key, slot in (("slot1", 1), ("slot0", 0), ("slot2", 2)):
        for f, v in e.get(key, {}).items():
            if f == "log":  # in Index order from the dummy (the engine's ring, include/mraft.h)
                h = int(st["log_head"][slot]) if "log_head" in st else 0
                got = [st["log_term"][slot * L + (h + j) % L] for j in range(len(v))]
                assert got == v, (k["name"], got, v)
            else:
                assert st[f][slot] == v, (k["name"], f, st[f][slot], v)
    if "flags" in e:
        assert list(out["flags"]) == e["flags"], (k["name"], out["flags"], e["flags"])
    if "next0" in e:
        assert list(st["next_index"][0:P]) == e["next0"], k["name"]
        assert list(st["match_index"][0:P]) == e["match0"], k["name"]


def tick_vectors():
    """Seeded tick vectors: inputs from the synthetic generator, outputs from
    the Python restatement (independent of the C oracle under test)."""
    from multiraft_amd import synth_tick_state
    out = {}
    for i, (G, P, L) in enumerate([(24, 3, 32), (16, 5, 64), (12, 7, 48)]):
        st, lp, _ = synth_tick_state(G, P, L, seed=0x5EED + i, nthreads=1)
        pst, gf = po.replicate_tick(st, G, P, L, lp)
        out[f"v{i}_dims"] = np.array([G, P, L], dtype=np.int32)
        out[f"v{i}_leader_peer"] = lp
        for kk, v in st.items():
            out[f"v{i}_in_{kk}"] = v
        for kk, v in pst.items():
            out[f"v{i}_out_{kk}"] = v.astype(np.int32)
        out[f"v{i}_flags"] = gf
    return out


BIN_ARRAYS = ("current_term", "voted_for", "state", "commit_index", "last_applied", "dummy_index",
              "last_index", "granted_votes", "log_term", "match_index", "next_index", "persist_dirty")


def tick_vectors_bin(z) -> bytes:
    """The tick vectors as the flat little-endian int32 file the plain-C host
    test reads (tests/c_host/mraft_host_tick.c): "MRTV", version 1, count;
    per vector G, P, L, leader_peer[G], group flags[G], the GetState words
    of every group's leader replica (replica 0 when leader_peer is out of
    range, include/mraft.h mraft_replicate_tick_export) commit[G] and
    term<<1|isLeader[G], then the BIN_ARRAYS inputs and the expected outputs."""
    parts = [b"MRTV"]
    n = 0
    while f"v{n}_dims" in z:
        n += 1
    parts.append(np.array([1, n], dtype="<i4").tobytes())
    for i in range(n):
        G, P, L = (int(x) for x in z[f"v{i}_dims"])
        lp = np.asarray(z[f"v{i}_leader_peer"], dtype=np.int64)
        rep = np.where((lp >= 0) & (lp < P), lp, 0) + np.arange(G) * P
        out = {k: np.asarray(z[f"v{i}_out_{k}"], dtype=np.int64) for k in BIN_ARRAYS}
        commit = out["commit_index"][rep]
        tl = (out["current_term"][rep] << 1) | (out["state"][rep] == 1)
        vec = [z[f"v{i}_dims"], z[f"v{i}_leader_peer"], z[f"v{i}_flags"], commit, tl]
        vec += [z[f"v{i}_in_{k}"] for k in BIN_ARRAYS] + [z[f"v{i}_out_{k}"] for k in BIN_ARRAYS]
        parts += [np.ascontiguousarray(a, dtype="<i4").tobytes() for a in vec]
    return b"".join(parts)


if __name__ == "__main__":
    kats = build()
    for k in kats:
        check_kat(k, run_py(k))
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kats, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "tick_vectors.npz"), **tick_vectors())
    with open(os.path.join(HERE, "tick_vectors.bin"), "wb") as f:
        f.write(tick_vectors_bin(np.load(os.path.join(HERE, "tick_vectors.npz"))))
    print(f"wrote {len(kats)} KATs and tick vectors")
