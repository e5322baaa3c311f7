"""The engine's Index domain on the CPU oracle (include/mraft.h: Raft Indexes
up to 2^31 - 2; Go's int is 64-bit, the engine's int32). The reference's
decisions depend on Index differences only (src/raft/raft_append_entry.go:
prevLogIndex / nextIndex / ConflictIndex arithmetic, the matchIndex order
statistic), so a step on a state whose every Index is moved up by `off`
equals the step on the original with its Index outputs moved up by `off`.
Checked here at the top of the domain for the tick, the message path (by
reference, host buffers, rings of stale leaders) and against the Python
restatement (arbitrary-precision integers) — the property the GPU tests
(test_index_domain_gpu.py, test_message_path_gpu.py) rely on at the same
Indexes — and the two engine limits just past the domain: an AppendEntries
whose last entry would be Index 2^31 - 1 is malformed (MRAFT_ITEM_BAD_SLOT) and
a Start that would append there is MRAFT_ITEM_LOG_FULL."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

import pyoracle as po  # noqa: E402
from message_cases import (all_follower_items, external_entries, results_of, shift_indices,  # noqa: E402
                           stale_cycle_state, top_offset)
from oracle_lib import Oracle, assert_states_equal  # noqa: E402

from multiraft_amd import synth_tick_state  # noqa: E402
from multiraft_amd._abi import AE_REPLY, IS_ARGS  # noqa: E402

TOP = 2**31 - 2


@pytest.mark.parametrize("j", [0, 7])
def test_tick_shift_invariance_at_top(j):
    G, P, L = 64, 5, 128
    st0, lp, _ = synth_tick_state(G, P, L, seed=500 + j, nthreads=1)
    off = top_offset(st0, j)
    assert off > 2**30
    st = shift_indices(st0, off)
    a, b = Oracle(G, P, L, st0), Oracle(G, P, L, st)
    ga, gb = a.replicate_tick(lp), b.replicate_tick(lp)
    assert np.array_equal(ga, gb)
    assert_states_equal(shift_indices(a.state(), off), b.state(), G, P, L, "shifted tick")
    # the Python restatement (unbounded ints) on the shifted state
    pst, pgf = po.replicate_tick(st, G, P, L, lp)
    assert np.array_equal(gb, pgf)
    assert_states_equal(b.state(), pst, G, P, L, "shifted tick vs Python restatement")
    assert (ga & 2).any()


@pytest.mark.parametrize("mode", ["reference", "host", "cycles"])
def test_message_path_shift_invariance_at_top(mode):
    G, P, L = 48, 5, 128
    rng = np.random.default_rng(510)
    st0, lp, _ = synth_tick_state(G, P, L, seed=511, nthreads=1)
    if mode == "cycles":
        st0, slots, peers = stale_cycle_state(st0, lp, G, P, L, rng, range(0, G, 2), 3)
    else:
        slots, peers = all_follower_items(lp, G, P)
    off = top_offset(st0, 2)
    outs = []
    for st in (st0, shift_indices(st0, off)):
        o = Oracle(G, P, L, st)
        args, gerr = o.gather_append_args(slots, peers)
        ok = gerr == 0
        if mode == "host":
            a2, buf = external_entries(args, ok, st, L)
            a2 = a2[ok]
            rep, herr = o.handle_append_entries(a2, buf)
            args, sl, pe = args[ok], slots[ok], peers[ok]
        else:
            rep, herr = o.handle_append_entries(args, None)
            sl, pe = slots, peers
        res, seg = results_of(sl, pe, args, rep, herr, G, P)
        f, ferr = o.process_append_replies(res, seg)
        outs.append((args, rep, herr, f, ferr, o.state()))
    (a0, r0, h0, f0, e0, s0), (a1, r1, h1, f1, e1, s1) = outs
    assert np.array_equal(h0, h1) and np.array_equal(f0, f1) and np.array_equal(e0, e1)
    assert (h0 == 0).any() and (r0["success"] == 1).any()
    # Index fields move by off; every other field is equal
    assert np.array_equal(a1["prev_log_index"].astype(np.int64), a0["prev_log_index"].astype(np.int64) + off)
    assert np.array_equal(a1["leader_commit"].astype(np.int64), a0["leader_commit"].astype(np.int64) + off)
    for k in ("term", "prev_log_term", "n_entries", "flags", "slot"):
        assert np.array_equal(a0[k], a1[k]), k
    ci0, ci1 = r0["conflict_index"].astype(np.int64), r1["conflict_index"].astype(np.int64)
    has_ci = ci0 != 0
    assert np.array_equal(ci1[has_ci], ci0[has_ci] + off) and not ci1[~has_ci].any()
    for k in ("term", "success"):
        assert np.array_equal(r0[k], r1[k]), k
    assert_states_equal(shift_indices(s0, off), s1, G, P, L, f"shifted message path ({mode})")


def test_past_the_index_domain_oracle():
    G, P, L = 8, 3, 32
    st0, lp, _ = synth_tick_state(G, P, L, seed=520, nthreads=1)
    st = shift_indices(st0, top_offset(st0, 0))
    o = Oracle(G, P, L, st)
    slots, peers = all_follower_items(lp, G, P)
    args, gerr = o.gather_append_args(slots, peers)
    a = args[gerr == 0].copy()
    a["n_entries"] = 2
    a["entries_offset"] = np.arange(len(a)) * 2
    a["prev_log_index"] = np.where(np.arange(len(a)) % 2 == 0, TOP - 2, TOP - 1)
    rep, herr = o.handle_append_entries(a, np.ones(2 * len(a), np.int32))
    bad = rep[1::2]
    assert (herr[1::2] == 6).all() and not (bad["term"].any() or bad["success"].any() or bad["conflict_index"].any())
    assert (herr[0::2] != 6).all()
    # the rejected half changed nothing: re-run only the accepted half on the original
    o2 = Oracle(G, P, L, st)
    o2.handle_append_entries(a[0::2], np.ones(2 * len(a), np.int32))
    assert_states_equal(o.state(), o2.state(), G, P, L, "malformed items change nothing")
    # Start: leaders whose last would pass 2^31 - 2
    ldr = np.array([g * P + int(lp[g]) for g in range(G) if lp[g] >= 0], np.int32)
    last = o.state()["last_index"][ldr].astype(np.int64)
    k = (TOP - last + 1).astype(np.int32)  # one past the top for every leader
    idx, term, isl, err = o.start(ldr, k)
    assert (err == 3).all() and (idx == -1).all()


def test_past_the_index_domain_fold_and_snapshot_oracle():
    """Reply records whose acknowledged entries would end past 2^31 - 2 (or
    with a negative count) make their segment malformed; an InstallSnapshot
    whose LastIncludedIndex is past it is malformed; everything else is
    folded / installed as usual."""
    G, P, L = 8, 3, 32
    st0, lp, _ = synth_tick_state(G, P, L, seed=521, nthreads=1)
    st = shift_indices(st0, top_offset(st0, 0))
    o = Oracle(G, P, L, st)
    slots, peers = all_follower_items(lp, G, P)
    args, gerr = o.gather_append_args(slots, peers)
    ok = gerr == 0
    res, seg = results_of(slots[ok], peers[ok], args[ok], np.zeros(int(ok.sum()), dtype=AE_REPLY),
                          np.zeros(int(ok.sum()), np.int32), G, P)
    res = res.copy()
    r0 = int(seg[0])
    res["args_n_entries"][r0] = TOP - int(res["args_prev_log_index"][r0]) + 1
    r1 = int(seg[1])
    res["args_n_entries"][r1] = -1
    f, ferr = o.process_append_replies(res, seg)
    assert (ferr[int(seg[0]):int(seg[2])] == 6).all() and not ferr[int(seg[2]):].any()
    ldr = np.array([g * P + int(lp[g]) for g in range(G) if lp[g] >= 0], np.int32)
    isa = np.zeros(len(ldr), dtype=IS_ARGS)
    isa["slot"], isa["term"], isa["leader_id"] = ldr, 1 << 20, (ldr + 1) % P
    isa["last_included_index"] = np.where(np.arange(len(ldr)) % 2 == 0, 2**31 - 1, TOP)
    isa["last_included_term"] = 3
    rep, fl, err = o.handle_install_snapshot(isa)
    assert (err[0::2] == 6).all() and (err[1::2] == 0).all() and (fl[1::2] != 0).all()
    assert (o.state()["dummy_index"][ldr[1::2]] == TOP).all()
