"""Index-domain cases shared by tests/test_index_domain_gpu.py (in process,
through libmraft_hip.so) and tests/test_bounds_debug_gpu.py (a subprocess on
the MRAFT_DEBUG_BOUNDS build, libmraft_hip_dbg.so, which counts every pass
dereference whose 32-bit ring offset is out of its valid range).

Every case moves a seeded state's Raft Indexes up so its highest Index sits
within 8 of the top of the engine's domain (2^31 - 2: nextIndex = Index + 1
must be an int32, include/mraft.h) and checks the GPU against the CPU oracle,
bit for bit, through the path named by the case: the fused tick, and the
message path (gather -> HandleAppendEntries -> reply fold,
src/raft/raft_append_entry.go:20-162) with entries from a host buffer
(aligned / misaligned: the flat-source pass), by reference in place, deferred
in place (a stale second leader), staged (rings of stale leaders within the
stage) and in the ordered fallback (stage capacity 0 and 64: the cycle buffer).
The batches carry MRAFT_AE_ENTRIES_SORTED where the leader's terms are sorted,
so the flag's first check (prevLogTerm <= entry 0, read through the source
before the pass) runs at those Indexes too: the read that faulted in round 5
(DESIGN.md §5, r5_v1)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
if os.path.dirname(HERE) not in sys.path:
    sys.path.insert(0, os.path.dirname(HERE))

from message_cases import (all_follower_items, external_entries, results_of, shift_indices,  # noqa: E402
                           stale_cycle_state, stale_second_leader_state, top_offset)
from oracle_lib import Oracle, assert_states_equal  # noqa: E402

from multiraft_amd import Engine, synth_tick_state  # noqa: E402
from multiraft_amd._abi import AE_REPLY, IS_ARGS  # noqa: E402

MSG_MODES = ("aligned", "misaligned", "reference", "deferred", "staged", "ordered", "ordered64")
TOP = 2**31 - 2


def tick_case(j: int, G: int = 96, P: int = 5, L: int = 256, seed: int = 404):
    """The fused tick with the highest Index at 2^31 - 2 - j: GPU == oracle,
    and the oracle's step equals the unshifted step shifted (Index-difference
    invariance)."""
    st0, lp, _ = synth_tick_state(G, P, L, seed=seed + j)
    off = top_offset(st0, j)
    st = shift_indices(st0, off)
    assert max(int(st["last_index"].max()), int(st["next_index"].max()) - 1) == TOP - j
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        gf = e.replicate_tick(lp)
        got = e.store_state()
    ogf = o.replicate_tick(lp)
    assert np.array_equal(gf, ogf), f"tick j={j}: group flags"
    assert_states_equal(got, o.state(), G, P, L, f"tick j={j}")
    o0 = Oracle(G, P, L, st0)
    assert np.array_equal(o0.replicate_tick(lp), ogf)
    assert_states_equal(shift_indices(o0.state(), off), o.state(), G, P, L, f"tick j={j}: shift invariance")
    return int((gf & 2).astype(bool).sum())


def message_case(mode: str, j: int = 3, G: int = 96, P: int = 5, L: int = 256, seed: int = 405,
                 shift: bool = True):
    """gather -> HandleAppendEntries -> fold with the highest Index at
    2^31 - 2 - j, entries as `mode` says (module docstring). Returns the number
    of successful merges (the caller checks the case did merge)."""
    rng = np.random.default_rng(seed + j)
    st0, lp, _ = synth_tick_state(G, P, L, seed=seed + j)
    cap = None
    if mode == "deferred":
        st0, slots, peers = stale_second_leader_state(st0, lp, G, P, L, rng, range(0, G, 2))
    elif mode in ("staged", "ordered", "ordered64"):
        st0, slots, peers = stale_cycle_state(st0, lp, G, P, L, rng, range(0, G, 2), 2 if mode == "staged" else 3)
        cap = {"staged": None, "ordered": 0, "ordered64": 64}[mode]
    else:
        slots, peers = all_follower_items(lp, G, P)
    st = shift_indices(st0, top_offset(st0, j)) if shift else st0
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap is not None:
            e.set_stage_capacity(cap)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(gerr, ogerr) and np.array_equal(args, oargs), f"{mode}: gather"
        ok = gerr == 0
        # the sorted-terms claim rides on most merging messages (its first check reads
        # entry 0 through the source before the pass)
        assert ((args["flags"][ok] & 1) != 0).any(), f"{mode}: no sorted-terms flag in the batch"
        if mode in ("aligned", "misaligned"):
            a2, buf = external_entries(args, ok, st, L, misalign=(mode == "misaligned"))
            a2 = a2[ok]
            rep, herr, gres = e.handle_append_entries(a2, buf, results=True)
            orep, oherr = o.handle_append_entries(a2, buf)
            args, slots, peers = args[ok], slots[ok], peers[ok]
        else:
            rep, herr, gres = e.handle_append_entries(args, None, results=True)
            orep, oherr = o.handle_append_entries(args, None)
        assert np.array_equal(herr, oherr), f"{mode}: handle errors"
        assert np.array_equal(rep, orep), f"{mode}: replies"
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{mode}: after handle")
        res, seg = results_of(slots, peers, args, rep, herr, G, P)
        okh = herr == 0
        hand = gres[okh][np.argsort(gres["slot"][okh], kind="stable")]
        assert np.array_equal(hand, res), f"{mode}: handler's reply records"
        f, ferr = e.process_append_replies(res, seg)
        of, oferr = o.process_append_replies(res, seg)
        assert np.array_equal(ferr, oferr) and np.array_equal(f, of), f"{mode}: fold"
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{mode}: after fold")
    return int((rep["success"][herr == 0] == 1).sum())


def malformed_case(G: int = 16, P: int = 3, L: int = 64, seed: int = 406):
    """Past the domain: an AppendEntries whose last entry would be Index
    2^31 - 1 is malformed (MRAFT_ITEM_BAD_SLOT, no state change), one ending
    at 2^31 - 2 is handled; a Start that would append past 2^31 - 2 is
    MRAFT_ITEM_LOG_FULL, one that reaches it appends. GPU == oracle."""
    st0, lp, _ = synth_tick_state(G, P, L, seed=seed)
    ldr = np.array([g * P + int(lp[g]) for g in range(G) if lp[g] >= 0], np.int32)
    room = L - 1 - (st0["last_index"][ldr] - st0["dummy_index"][ldr])
    x = int(ldr[np.argmax(np.where(room >= 2, st0["last_index"][ldr], -1))])
    assert L - 1 - (st0["last_index"][x] - st0["dummy_index"][x]) >= 2
    # leader x's last at 2^31 - 3: Start of 1 then 1 more reaches the top, a third is past it
    off = (TOP - 1) - int(st0["last_index"][x])
    st = shift_indices(st0, min(off, top_offset(st0, 0)))
    off = min(off, top_offset(st0, 0))
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        slots, peers = all_follower_items(lp, G, P)
        args, gerr = e.gather_append_args(slots, peers)
        a = args[gerr == 0].copy()
        buf = np.arange(8 * len(a), dtype=np.int32) % 7 + 1
        a["entries_offset"] = np.arange(len(a)) * 8
        a["flags"] = 1
        # half end at the domain's top (last entry Index 2^31 - 2), half one past it
        a["n_entries"] = 2
        a["prev_log_index"] = np.where(np.arange(len(a)) % 2 == 0, TOP - 2, TOP - 1)
        rep, herr = e.handle_append_entries(a, buf)
        orep, oherr = o.handle_append_entries(a, buf)
        assert np.array_equal(herr, oherr) and np.array_equal(rep, orep), "malformed: handle"
        assert (herr[1::2] == 6).all(), "past the domain: MRAFT_ITEM_BAD_SLOT"
        assert_states_equal(e.store_state(), o.state(), G, P, L, "malformed: after handle")
        # reply records: every other segment holds one record whose entries would end
        # past the domain (or a negative count): the whole segment is malformed
        gargs, gerr = e.gather_append_args(slots, peers)
        oka = gerr == 0
        res, seg = results_of(slots[oka], peers[oka], gargs[oka],
                              np.zeros(int(oka.sum()), dtype=AE_REPLY), np.zeros(int(oka.sum()), np.int32), G, P)
        res = res.copy()
        for sgi in range(0, len(seg) - 1, 2):
            r0 = int(seg[sgi])
            if sgi % 4 == 0:
                res["args_n_entries"][r0] = TOP - int(res["args_prev_log_index"][r0]) + 1
            else:
                res["args_n_entries"][r0] = -1
        f, ferr = e.process_append_replies(res, seg)
        of, oferr = o.process_append_replies(res, seg)
        assert np.array_equal(ferr, oferr) and np.array_equal(f, of), "malformed: fold"
        assert (ferr[int(seg[0]):int(seg[1])] == 6).all()
        assert_states_equal(e.store_state(), o.state(), G, P, L, "malformed: after fold")
        # InstallSnapshot args past the domain
        isa = np.zeros(len(ldr), dtype=IS_ARGS)
        isa["slot"] = ldr
        isa["term"] = 1 << 20
        isa["leader_id"] = (ldr + 1) % P
        isa["last_included_index"] = np.where(np.arange(len(ldr)) % 2 == 0, 2**31 - 1, TOP)
        isa["last_included_term"] = 3
        for x_ in zip(e.handle_install_snapshot(isa), o.handle_install_snapshot(isa)):
            assert np.array_equal(*x_), "malformed: InstallSnapshot"
        assert_states_equal(e.store_state(), o.state(), G, P, L, "malformed: after InstallSnapshot")
        for k in (1, 2, 1):
            r = e.start(np.array([x], np.int32), np.array([k], np.int32))
            orr = o.start(np.array([x], np.int32), np.array([k], np.int32))
            for u, v in zip(r, orr):
                assert np.array_equal(u, v), f"malformed: Start {k}"
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"malformed: after Start {k}")
        if off == (TOP - 1) - int(st0["last_index"][x]):
            # x was at 2^31 - 3: the first Start reached 2^31 - 2, the second is past it, the third too
            assert int(o.state()["last_index"][x]) == TOP


def main():
    """Every case on the library MRAFT_LIB names (the bounds-checking build),
    then its violation counters: one JSON line."""
    from multiraft_amd import _abi
    lib = _abi.lib()
    out = {"cases": [], "violations": {}}
    for j in (0, 5):
        out["cases"].append(["tick", j, tick_case(j)])
    for m in MSG_MODES:
        out["cases"].append([m, 3, message_case(m)])
    # the same paths at ordinary Indexes (the synth generator's own)
    for m in ("aligned", "reference", "ordered"):
        out["cases"].append([m + "_low", message_case(m, shift=False, seed=407)])
    malformed_case()
    for fn in ("mraft_debug_bounds_kernels", "mraft_debug_bounds_tick"):
        f = getattr(lib, fn)
        f.restype = __import__("ctypes").c_longlong
        f.argtypes = [__import__("ctypes").c_int]
        out["violations"][fn] = int(f(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
