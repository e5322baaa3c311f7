"""CPU tests: the oracle against the committed known-answer tests and tick
vectors, and the C restatement against the independent Python restatement on
seeded random states (no GPU)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

import pyoracle as po  # noqa: E402
from kat_runner import kat_state, load_kats, run_kat  # noqa: E402
from make_golden import check_kat, run_py  # noqa: E402
from oracle_lib import terms_sorted_exact, Oracle, assert_states_equal  # noqa: E402

from multiraft_amd import synth_fold_batch, synth_tick_state  # noqa: E402
from multiraft_amd._abi import AE_ARGS, RV_ARGS, RV_RESULT  # noqa: E402

KATS = load_kats()


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_kat_c_oracle(k):
    o = Oracle(k["G"], k["P"], k["L"], kat_state(k))
    check_kat(k, run_kat(k, o, o.state))


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_kat_py_oracle(k):
    check_kat(k, run_py(k))


def test_tick_vectors_c_oracle():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "tick_vectors.npz"))
    i = 0
    while f"v{i}_dims" in z:
        G, P, L = (int(x) for x in z[f"v{i}_dims"])
        st = {k[len(f"v{i}_in_"):]: z[k] for k in z.files if k.startswith(f"v{i}_in_")}
        exp = {k[len(f"v{i}_out_"):]: z[k] for k in z.files if k.startswith(f"v{i}_out_")}
        o = Oracle(G, P, L, st)
        gf = o.replicate_tick(z[f"v{i}_leader_peer"])
        assert np.array_equal(gf, z[f"v{i}_flags"])
        assert_states_equal(o.state(), exp, G, P, L, f"vector {i}")
        i += 1
    assert i >= 3


def test_synth_matches_fixture_inputs():
    """The generator is deterministic: regenerating the fixture inputs gives
    the committed arrays bit for bit."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "tick_vectors.npz"))
    for i in range(3):
        G, P, L = (int(x) for x in z[f"v{i}_dims"])
        st, lp, _ = synth_tick_state(G, P, L, seed=0x5EED + i, nthreads=1)
        assert np.array_equal(lp, z[f"v{i}_leader_peer"])
        for k, v in st.items():
            if k in ("log_head", "has_snapshot") and f"v{i}_in_{k}" not in z.files:
                assert not v.any()  # fixture made before these arrays: all zero
                continue
            if k == "terms_sorted" and f"v{i}_in_{k}" not in z.files:
                # fixture made before this array: it is the logs' own sortedness
                fx = {kk: z[f"v{i}_in_{kk}"] for kk in ("log_term", "dummy_index", "last_index")}
                fx["log_head"] = np.zeros(G * P, np.int32)
                assert np.array_equal(v, terms_sorted_exact(fx, G, P, L))
                continue
            assert np.array_equal(v, z[f"v{i}_in_{k}"]), k


@pytest.mark.parametrize("G,P,L,seed", [(48, 3, 64, 1), (32, 5, 128, 2), (24, 7, 96, 3),
                                        (40, 2, 32, 4), (30, 4, 16, 5), (16, 8, 64, 6),
                                        (20, 1, 16, 7), (64, 5, 8, 8)])
def test_tick_c_vs_py(G, P, L, seed):
    st, lp, _ = synth_tick_state(G, P, L, seed=seed, nthreads=1)
    lp = lp.copy()
    lp[::7] = -1          # idle groups
    if G > 9 and P > 1:
        lp[9] = P         # bad leader index -> error
    o = Oracle(G, P, L, st)
    gf = o.replicate_tick(lp)
    pst, pgf = po.replicate_tick(st, G, P, L, lp)
    assert np.array_equal(gf, pgf)
    assert_states_equal(o.state(), pst, G, P, L, "tick")


def test_tick_mt_equals_st():
    G, P, L = 512, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=11)
    a, b = Oracle(G, P, L, st), Oracle(G, P, L, st)
    assert np.array_equal(a.replicate_tick(lp), b.replicate_tick(lp, nthreads=8))
    assert_states_equal(a.state(), b.state(), G, P, L, "mt")


def test_tick_count_invariants():
    G, P, L = 256, 5, 512
    st, lp, _ = synth_tick_state(G, P, L, seed=12)
    o = Oracle(G, P, L, st)
    r, w, act = o.replicate_tick_count(lp)
    assert act == G and r > 0 and w > 0
    # counting never changes the oracle's own state
    assert_states_equal(o.state(), st, G, P, L, "count is side-effect free")


def test_fold_batch_c_vs_py():
    G, P, L = 128, 5, 64
    st, lp, _ = synth_tick_state(G, P, L, seed=21)
    items, seg = synth_fold_batch(st, G, P, L, lp, seed=22)
    o = Oracle(G, P, L, st)
    flags, err = o.process_append_replies(items, seg)
    assert not err.any()
    rafts = po.from_soa(st, G, P, L)
    pflags = []
    for it in items:
        rf = rafts[it["slot"]]
        args = po.AppendEntriesArgs(Term=int(it["args_term"]), LeaderId=rf.me,
                                    Entries=[None] * int(it["args_n_entries"]),
                                    PrevLogIndex=int(it["args_prev_log_index"]), PrevLogTerm=0,
                                    LeaderCommit=0)
        rep = po.AppendEntriesReply(Term=int(it["reply_term"]), Success=bool(it["reply_success"]),
                                    ConflictIndex=int(it["reply_conflict_index"]))
        pflags.append(rf.processAppendEntriesReply(int(it["peer"]), args, rep))
    assert flags.tolist() == pflags
    assert_states_equal(o.state(), po.to_soa(rafts, st, G, P, L), G, P, L, "fold")


def test_fold_long_segments_c_vs_py():
    """Segments of up to 150 replies in arrival order (repeated peers, stale
    and higher terms, a1 evaluated many times per segment): C oracle ==
    Python restatement, flags and state."""
    from oracle_lib import random_reply_segments
    G, P, L = 48, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=23)
    items, seg = random_reply_segments(st, G, P, lp, seed=24)
    assert (np.diff(seg) > 64).any()
    o = Oracle(G, P, L, st)
    flags, err = o.process_append_replies(items, seg)
    assert not err.any()
    rafts = po.from_soa(st, G, P, L)
    pflags = []
    for it in items:
        rf = rafts[it["slot"]]
        args = po.AppendEntriesArgs(Term=int(it["args_term"]), LeaderId=rf.me,
                                    Entries=[None] * int(it["args_n_entries"]),
                                    PrevLogIndex=int(it["args_prev_log_index"]), PrevLogTerm=0,
                                    LeaderCommit=0)
        rep = po.AppendEntriesReply(Term=int(it["reply_term"]), Success=bool(it["reply_success"]),
                                    ConflictIndex=int(it["reply_conflict_index"]))
        pflags.append(rf.processAppendEntriesReply(int(it["peer"]), args, rep))
    assert flags.tolist() == pflags
    assert ((flags & 2) != 0).sum() > 10  # COMMITTED on many replies
    assert_states_equal(o.state(), po.to_soa(rafts, st, G, P, L), G, P, L, "fold long")


def test_item_path_equals_tick():
    """gather (a3) -> handle (a4) -> process (a2+a1) through the item-level
    oracle entry points equals the fused tick."""
    G, P, L = 64, 5, 128
    st, lp, _ = synth_tick_state(G, P, L, seed=31)
    fused = Oracle(G, P, L, st)
    fused.replicate_tick(lp)
    o = Oracle(G, P, L, st)
    slots = np.array([g * P + lp[g] for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    peers = np.array([p for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    args, gerr = o.gather_append_args(slots, peers)
    ok = gerr == 0
    rep, herr = o.handle_append_entries(args[ok], None)
    from multiraft_amd._abi import AE_RESULT
    res = np.zeros(int(ok.sum()), dtype=AE_RESULT)
    res["slot"] = slots[ok]
    res["peer"] = peers[ok]
    res["args_term"] = args["term"][ok]
    res["args_prev_log_index"] = args["prev_log_index"][ok]
    res["args_n_entries"] = args["n_entries"][ok]
    res["reply_term"] = rep["term"]
    res["reply_success"] = rep["success"]
    res["reply_conflict_index"] = rep["conflict_index"]
    keep = herr == 0
    res = res[keep]
    seg = np.concatenate([[0], np.cumsum(np.bincount(res["slot"] // P, minlength=G))]).astype(np.int64)
    o.process_append_replies(res, seg)
    assert_states_equal(o.state(), fused.state(), G, P, L, "item path vs fused")


def _random_vote_state(G, P, L, seed):
    rng = np.random.default_rng(seed)
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    # scramble votes / terms so every branch of HandleRequestVote is exercised
    st["voted_for"][:] = rng.integers(-1, P, size=G * P)
    st["current_term"][:] = rng.integers(1, 6, size=G * P)
    last = rng.integers(0, 8, size=G * P)
    st["last_index"][:] = last
    st["dummy_index"][:] = 0
    lt = st["log_term"].reshape(G * P, L)
    lt[:, :] = 0
    for s in range(G * P):
        lt[s, 1:last[s] + 1] = np.sort(rng.integers(1, 5, size=last[s]))
    return st


def test_elections_c_vs_py():
    G, P, L = 64, 5, 16
    rng = np.random.default_rng(5)
    st = _random_vote_state(G, P, L, 41)
    o = Oracle(G, P, L, st)
    rafts = po.from_soa(st, G, P, L)
    cands = np.array([g * P + rng.integers(0, P) for g in range(G)], np.int32)
    args, err = o.start_election(cands)
    pargs = [rafts[c].StartElection() for c in cands]
    assert [int(a) for a in args["term"]] == [a.Term for a in pargs]
    # every other peer votes
    rv = np.zeros(G * (P - 1), dtype=RV_ARGS)
    res = np.zeros(G * (P - 1), dtype=RV_RESULT)
    i = 0
    for g, c in enumerate(cands):
        for p in range(P):
            v = g * P + p
            if v == c:
                continue
            a = args[g].copy()
            if rng.random() < 0.2:
                a["last_log_term"] = rng.integers(0, 6)
            rv[i] = (v, a["candidate_id"], a["term"], a["last_log_index"], a["last_log_term"])
            res[i] = (c, p, a["term"], 0, 0)
            i += 1
    rep, rerr = o.handle_request_vote(rv)
    assert not rerr.any()
    for j in range(len(rv)):
        r = po.RequestVoteReply()
        rafts[rv["slot"][j]].HandleRequestVote(po.RequestVoteArgs(
            CandidateId=int(rv["candidate_id"][j]), Term=int(rv["term"][j]),
            LastLogIndex=int(rv["last_log_index"][j]), LastLogTerm=int(rv["last_log_term"][j])), r)
        assert (r.Term, int(r.VoteGranted)) == (int(rep["term"][j]), int(rep["vote_granted"][j]))
    res["reply_term"] = rep["term"]
    res["vote_granted"] = rep["vote_granted"]
    seg = np.arange(0, len(res) + 1, P - 1, dtype=np.int64)
    flags, ferr = o.process_vote_replies(res, seg)
    assert not ferr.any()
    pflags = []
    for j in range(len(res)):
        c = int(res["slot"][j])
        pflags.append(rafts[c].tally(po.RequestVoteArgs(CandidateId=c % P, Term=int(res["args_term"][j]),
                                                        LastLogIndex=0, LastLogTerm=0),
                                     po.RequestVoteReply(Term=int(res["reply_term"][j]),
                                                         VoteGranted=bool(res["vote_granted"][j]))))
    assert flags.tolist() == pflags
    assert_states_equal(o.state(), po.to_soa(rafts, st, G, P, L), G, P, L, "elections")


def test_dup_slots_rejected():
    G, P, L = 4, 3, 16
    st, lp, _ = synth_tick_state(G, P, L, seed=51)
    o = Oracle(G, P, L, st)
    a = np.zeros(3, dtype=AE_ARGS)
    a["slot"] = [1, 1, 99]
    a["term"] = 1
    rep, err = o.handle_append_entries(a, np.zeros(4, np.int32))
    assert err.tolist() == [0, 5, 6]


@pytest.mark.parametrize("P,L,mono", [(2, 8, False), (3, 16, False), (5, 12, False), (5, 16, True),
                                      (7, 10, False), (8, 9, False), (4, 64, False)])
def test_tick_random_adversarial_c_vs_py(P, L, mono):
    from random_states import random_tick_state
    rng = np.random.default_rng(1000 + P * 100 + L)
    G = 300
    st, lp = random_tick_state(rng, G, P, L, monotone=mono)
    o = Oracle(G, P, L, st)
    gf = o.replicate_tick(lp)
    pst, pgf = po.replicate_tick(st, G, P, L, lp)
    assert np.array_equal(gf, pgf)
    assert_states_equal(o.state(), pst, G, P, L, "random tick")
    # every branch is exercised
    for bit in (1, 2, 4, 8, 16, 64):
        assert (gf & bit).any() or bit in (8, 64), bit


@pytest.mark.parametrize("P,L", [(2, 8), (3, 16), (5, 12), (5, 256), (8, 40)])
def test_tick_snapshot_heavy_c_vs_py(P, L):
    """Fused tick with the InstallSnapshot branch in most groups
    (raft_append_entry.go:27-34 -> raft_snapshot.go:15-69)."""
    from random_states import random_tick_state
    rng = np.random.default_rng(1500 + P * 100 + L)
    G = 300
    st, lp = random_tick_state(rng, G, P, L, snap=True)
    o = Oracle(G, P, L, st)
    gf = o.replicate_tick(lp)
    pst, pgf = po.replicate_tick(st, G, P, L, lp)
    assert np.array_equal(gf, pgf)
    assert_states_equal(o.state(), pst, G, P, L, "snapshot-heavy tick", heads=False)
    assert (gf & 8).any() and (gf & 256).any()


def _py_election_rounds(st, G, P, L, mask):
    rafts = po.from_soa(st, G, P, L)
    gf = np.zeros(G, np.int32)
    for g in range(G):
        for r in range(mask.shape[0]):
            m = int(mask[r, g])
            cands = [p for p in range(P) if (m >> p) & 1 and rafts[g * P + p].state != po.LEADER]
            args = {c: rafts[g * P + c].StartElection() for c in cands}
            reps = {}
            for v in range(P):
                for c in cands:
                    if c != v:
                        rep = po.RequestVoteReply()
                        rafts[g * P + v].HandleRequestVote(args[c], rep)
                        reps[(c, v)] = rep
            for c in cands:
                for v in range(P):
                    if c != v:
                        fl = rafts[g * P + c].tally(args[c], reps[(c, v)])
                        if fl & po.F_BECAME_LEADER:
                            gf[g] |= 128
                        if fl & po.F_STEPPED_DOWN:
                            gf[g] |= po.G_STEPPED_DOWN
    return po.to_soa(rafts, st, G, P, L), gf


@pytest.mark.parametrize("P", [3, 5, 7, 8])
def test_election_rounds_c_vs_py(P):
    from multiraft_amd import synth_election_state
    G, L, R = 96, 8, 12
    st, mask = synth_election_state(G, P, L, seed=90 + P, rounds=R, nthreads=1)
    o = Oracle(G, P, L, st)
    gf = o.election_rounds(mask)
    pst, pgf = _py_election_rounds(st, G, P, L, mask)
    assert np.array_equal(gf, pgf)
    assert_states_equal(o.state(), pst, G, P, L, "election rounds")
    assert (gf & 128).any() and (gf & 4).any()


def _py_snapshot_scenario(st, G, P, L, lp, seed):
    """The same scenario on the Python restatement (object model)."""
    from multiraft_amd._abi import IS_ARGS
    rng = np.random.default_rng(seed)
    rafts = po.from_soa(st, G, P, L)
    last, dummy = st["last_index"], st["dummy_index"]
    idx = np.minimum(dummy + rng.integers(-1, 6, size=G * P), last).astype(np.int32)
    bump = rng.random(G * P) < 0.05
    idx[bump] = last[bump] + 1  # index > lastIndex: sliceFrom panics in Go
    snap_err = np.array([rafts[s].Snapshot(int(idx[s])) for s in range(G * P)], np.int32)
    pairs = [(g * P + lp[g], p) for g in range(G) for p in range(P) if p != lp[g] and lp[g] >= 0]
    args = {}
    for (ld, p) in pairs:
        rf = rafts[ld]
        if rf.state == po.LEADER and rf.nextIndex[p] - 1 < rf.raftLog.dummyIndex():
            args[(ld, p)] = rf.gatherInstallSnapshot()
    reps, fls, errs = {}, {}, {}
    for (ld, p), a in args.items():
        rep = po.InstallSnapshotReply()
        fr = rafts[(ld // P) * P + p]
        if po._is_would_panic(fr, a):
            errs[(ld, p)] = 2
            reps[(ld, p)], fls[(ld, p)] = rep, 0
            continue
        inst = fr.HandleInstallSnapshot(a, rep)
        errs[(ld, p)] = 0
        reps[(ld, p)], fls[(ld, p)] = rep, (32 if inst else 0)
    prfl = []
    for (ld, p) in sorted([k for k in args if errs[k] == 0], key=lambda t: t[0]):
        prfl.append(rafts[ld].processInstallSnapshotReply(p, args[(ld, p)], reps[(ld, p)]))
    return snap_err, po.to_soa(rafts, st, G, P, L), [fls[k] for k in args], prfl, [errs[k] for k in args]


@pytest.mark.parametrize("P,L", [(3, 16), (5, 12), (7, 32)])
def test_snapshot_install_c_vs_py(P, L):
    from random_states import random_tick_state
    from snapshot_cases import run_snapshot_scenario
    G = 200
    rng = np.random.default_rng(500 + P)
    st, lp = random_tick_state(rng, G, P, L)
    lp = np.where((lp >= 0) & (lp < P), lp, 0).astype(np.int32)
    o = Oracle(G, P, L, st)
    out = run_snapshot_scenario(o, st, G, P, L, lp, seed=7)
    snap_err, pst, fls, prfl, errs = _py_snapshot_scenario(st, G, P, L, lp, seed=7)
    assert np.array_equal(out["snap_err"], snap_err)
    assert out["is_fl"].tolist() == fls
    assert out["is_herr"].tolist() == errs
    assert out["pr_fl"].tolist() == prfl
    assert_states_equal(o.state(), pst, G, P, L, "snapshot scenario", heads=False)
    assert (out["is_fl"] == 32).any() and (snap_err == 1).any()


def test_goshaped_tick_equals_oracle():
    """The CPU baseline's Go-shaped restatement (int64 structs, 40-B Entry
    slices, per-message copies) computes the same tick as the SoA oracle."""
    from oracle_lib import GoShaped
    for (G, P, L, seed) in [(256, 5, 256, 3), (128, 3, 512, 4), (64, 7, 128, 5)]:
        st, lp, _ = synth_tick_state(G, P, L, seed=seed)
        o = Oracle(G, P, L, st)
        o.replicate_tick(lp)
        gsh = GoShaped(G, P, L, st)
        assert gsh.replicate_tick(lp, nthreads=4) == 0
        got = gsh.state()
        exp = o.state()
        for k in exp:
            if k in ("persist_dirty", "log_term"):
                continue
            assert np.array_equal(got[k], exp[k]), k
        assert_states_equal({k: v for k, v in got.items() if k != "persist_dirty"},
                            {k: v for k, v in exp.items() if k != "persist_dirty"}, G, P, L, "go-shaped")


def test_goshaped_reset_restores():
    from oracle_lib import GoShaped
    G, P, L = 64, 5, 128
    st, lp, _ = synth_tick_state(G, P, L, seed=9)
    g = GoShaped(G, P, L, st)
    g.replicate_tick(lp, nthreads=2)
    first = g.state()
    g.reset(nthreads=3)
    assert_states_equal({k: v for k, v in g.state().items() if k != "persist_dirty"},
                        {k: v for k, v in st.items() if k != "persist_dirty"}, G, P, L, "reset")
    g.replicate_tick(lp, nthreads=1)
    assert_states_equal(g.state(), first, G, P, L, "re-run")


def test_election_rounds_mt_equals_st():
    from multiraft_amd import synth_election_state
    G, P, L, R = 512, 7, 16, 8
    st, mask = synth_election_state(G, P, L, seed=13, rounds=R)
    a, b = Oracle(G, P, L, st), Oracle(G, P, L, st)
    assert np.array_equal(a.election_rounds(mask), b.election_rounds(mask, nthreads=6))
    assert_states_equal(a.state(), b.state(), G, P, L, "election mt")


def test_handle_by_reference_stages_entries():
    """Entries by reference into the engine's log (entry_terms NULL): every
    item sees the log as it was when the batch was gathered (appendOneRound
    copies args.Entries, raft_append_entry.go:50-54), also when another item
    of the batch rewrites its source row (a stale second leader: lp -> q and
    q -> r in one batch)."""
    from message_cases import external_entries, stale_second_leader_state
    G, P, L = 48, 5, 64
    rng = np.random.default_rng(5)
    st, lp, _ = synth_tick_state(G, P, L, seed=91)
    st, slots, peers = stale_second_leader_state(st, lp, G, P, L, rng, range(0, G, 3))
    a = Oracle(G, P, L, st)
    b = Oracle(G, P, L, st)
    args, gerr = a.gather_append_args(slots, peers)
    assert (gerr == 0).all()
    rep, herr = a.handle_append_entries(args, None)
    a2, buf = external_entries(args, gerr == 0, st, L, misalign=False)
    rep2, herr2 = b.handle_append_entries(a2, buf)
    assert np.array_equal(herr, herr2) and np.array_equal(rep, rep2)
    assert_states_equal(a.state(), b.state(), G, P, L, "staged vs copied entries")
    # the batch does rewrite rows it also reads: q's row changed under lp -> q
    q_rows = slots[1::2]
    assert not np.array_equal(a.state()["log_term"].reshape(G * P, L)[q_rows],
                              st["log_term"].reshape(G * P, L)[q_rows])
