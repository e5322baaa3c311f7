"""terms_sorted, the engine's per-replica proof that the terms after the dummy
never decrease (include/mraft.h MRAFT_TERMS_SORTED), which lets a1
(advanceCommitIndexForLeader, src/raft/raft_append_entry.go:89-105) decide a
range by its top term instead of Go's downward loop.

Hand-built cases for every rule (the gather's args flag, the follower's
append, Start, InstallSnapshot's new log, restore, load) on the oracle and —
marked gpu — on libmraft_hip.so; the proof is checked sound (1 only over
sorted terms) wherever states are compared (tests/oracle_lib.py), and the
decisions with the proof withheld (all 0: Go's loop everywhere) equal the
decisions with it."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal, assert_terms_sorted_sound, terms_sorted_exact

from multiraft_amd import Engine, new_state, synth_fold_batch, synth_seed, synth_tick_state
from multiraft_amd._abi import AE_ARGS, LEADER, FOLLOWER

G, P, L = 4, 3, 16


def _oracle(st):
    return Oracle(G, P, L, st)


def _gpu(st):
    e = Engine(G, P, L)
    e.load_state(st)
    return e


BACKENDS = [pytest.param(_oracle, id="oracle"), pytest.param(_gpu, id="gpu", marks=pytest.mark.gpu)]


def _set_log(st, slot, terms, dummy=0):
    """Replica `slot`'s log = [dummy entry term, entries...] from Index dummy."""
    st["log_term"][slot * L:slot * L + len(terms)] = terms
    st["dummy_index"][slot] = dummy
    st["last_index"][slot] = dummy + len(terms) - 1
    st["commit_index"][slot] = dummy
    st["last_applied"][slot] = dummy


def _state():
    st = new_state(G, P, L)
    for g in range(G):
        ld = g * P
        st["state"][ld] = LEADER
        st["current_term"][ld] = 3
        for p in range(1, P):
            st["current_term"][ld + p] = 3
            st["state"][ld + p] = FOLLOWER
    return st


def _store(e):
    return e.store_state()


@pytest.mark.parametrize("mk", BACKENDS)
def test_gather_flag(mk):
    """mraft_gather_append_args sets MRAFT_AE_ENTRIES_SORTED when
    (prevLogTerm, entries...) never decrease: the leader's proof, with the
    dummy's own term compared when prev is the dummy."""
    st = _state()
    _set_log(st, 0, [0, 1, 1, 2, 3])          # group 0: sorted, dummy term 0
    _set_log(st, 3, [5, 1, 1, 2, 3])          # group 1: sorted after a dummy of term 5
    _set_log(st, 6, [0, 2, 1, 2, 3])          # group 2: not sorted
    _set_log(st, 9, [0, 1, 2])                # group 3: sorted, heartbeat
    for g, nx in ((0, (3, 1)), (1, (3, 1)), (2, (3, 1)), (3, (3, 3))):
        st["next_index"][g * P * P + 1] = nx[0]
        st["next_index"][g * P * P + 2] = nx[1]
    e = mk(st)
    assert list(_store(e)["terms_sorted"][::P]) == [1, 1, 0, 1]
    slots = np.repeat(np.arange(G) * P, 2).astype(np.int32)
    peers = np.tile([1, 2], G).astype(np.int32)
    args, err = e.gather_append_args(slots, peers)
    assert not err.any()
    #        g0: prev 2 > dummy, prev 0 (0 <= 1);  g1: prev 2, prev 0 (dummy term 5 > 1);
    #        g2: unsorted leader;  g3: n = 0 both
    assert list(args["flags"]) == [1, 1, 1, 0, 0, 0, 1, 1]


def _ae(slot, term, prev, prev_term, n, flags, commit=0):
    a = np.zeros(1, dtype=AE_ARGS)[0]
    a["slot"], a["term"], a["prev_log_index"], a["prev_log_term"] = slot, term, prev, prev_term
    a["n_entries"], a["flags"], a["leader_commit"], a["entries_offset"] = n, flags, commit, 0
    return a


@pytest.mark.parametrize("mk", BACKENDS)
def test_append_rule(mk):
    """HandleAppendEntries appending from Index k: terms_sorted becomes the
    args' flag when k - 1 is the dummy, is cleared without the flag, and is
    kept otherwise; no append, no change."""
    st = _state()
    _set_log(st, 1, [0, 1, 1, 1])             # sorted
    _set_log(st, 4, [0, 1, 1, 1])             # sorted
    _set_log(st, 7, [0, 3, 1, 1])             # not sorted
    _set_log(st, 10, [0, 1, 1, 1])            # sorted
    e = mk(st)
    assert list(_store(e)["terms_sorted"][[1, 4, 7, 10]]) == [1, 1, 0, 1]
    cases = [
        (_ae(1, 3, 1, 1, 3, 0), [1, 2, 2]),   # appends from 3 without the flag -> 0
        (_ae(4, 3, 1, 1, 3, 1), [1, 2, 2]),   # appends from 3 with it -> kept (1)
        (_ae(7, 3, 0, 0, 2, 1), [2, 2]),      # appends from 1 = dummy + 1 with it -> 1
        (_ae(10, 3, 0, 0, 2, 0), [1, 1]),     # every entry matches: no append, kept
    ]
    buf, args = [], []
    for a, ent in cases:
        a["entries_offset"] = len(buf)
        buf += ent
        args.append(a)
    rep, err = e.handle_append_entries(np.array(args, dtype=AE_ARGS), np.array(buf, np.int32))
    assert not err.any() and rep["success"].all()
    s = _store(e)
    assert list(s["terms_sorted"][[1, 4, 7, 10]]) == [0, 1, 1, 1]
    assert list(s["last_index"][[1, 4, 7, 10]]) == [4, 4, 2, 3]
    assert_terms_sorted_sound(s, G, P, L, "append rule")


@pytest.mark.parametrize("mk", BACKENDS)
def test_false_flag_is_not_honoured(mk):
    """MRAFT_AE_ENTRIES_SORTED crosses the network: a flag on
    entries that are not sorted — a descent among them, or prevLogTerm above
    the first — counts as no flag, so the follower's proof never claims an
    unsorted log (which a later a1 as leader would trust)."""
    st = _state()
    _set_log(st, 1, [0, 1, 1, 1])             # sorted
    _set_log(st, 4, [0, 2, 2, 2])             # sorted
    _set_log(st, 7, [0, 1, 1, 1])             # sorted
    _set_log(st, 10, [0, 1, 1, 1])            # sorted
    e = mk(st)
    assert list(_store(e)["terms_sorted"][[1, 4, 7, 10]]) == [1, 1, 1, 1]
    cases = [
        (_ae(1, 3, 1, 1, 3, 1), [1, 3, 2]),   # a descent after the first appended entry: not honoured -> 0
        (_ae(4, 3, 1, 2, 2, 1), [1, 1]),      # prevLogTerm 2 > entry 0: not honoured -> 0
        (_ae(7, 3, 0, 0, 3, 1), [2, 1, 1]),   # appends from dummy + 1, a descent: -> 0
        (_ae(10, 3, 1, 1, 3, 1), [1, 2, 3]),  # a true flag, append from 3: kept (1)
    ]
    buf, args = [], []
    for a, ent in cases:
        a["entries_offset"] = len(buf)
        buf += ent
        args.append(a)
    rep, err = e.handle_append_entries(np.array(args, dtype=AE_ARGS), np.array(buf, np.int32))
    assert not err.any() and rep["success"].all()
    s = _store(e)
    assert list(s["last_index"][[1, 4, 7, 10]]) == [4, 3, 3, 4]
    assert list(s["terms_sorted"][[1, 4, 7, 10]]) == [0, 0, 0, 1]
    assert_terms_sorted_sound(s, G, P, L, "false flags")


@pytest.mark.gpu
def test_false_flag_by_reference_gpu():
    """The same check on the by-reference message sets (one streaming pass per
    set, the flag checked on the pass's loads): args gathered from unsorted
    leaders with the flag forced on, on random adversarial states, rings
    rotated; GPU == oracle, proof sound."""
    from message_cases import all_follower_items, results_of
    from oracle_lib import rotate_rings
    from random_states import random_tick_state
    rng = np.random.default_rng(5)
    Gh, Ph, Lh = 256, 5, 96
    st, lp = random_tick_state(rng, Gh, Ph, Lh, monotone=False)
    st = rotate_rings(st, Gh, Ph, Lh, rng, 0.5)
    lpv = np.where((lp >= 0) & (lp < Ph), lp, -1).astype(np.int32)
    slots, peers = all_follower_items(lpv, Gh, Ph)
    o = Oracle(Gh, Ph, Lh, st)
    with Engine(Gh, Ph, Lh) as e:
        e.load_state(st)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr)
        ok = gerr == 0
        forged = args[ok].copy()
        forged["flags"] = 1
        rep, herr = e.handle_append_entries(forged, None)
        orep, oherr = o.handle_append_entries(forged, None)
        assert np.array_equal(rep, orep) and np.array_equal(herr, oherr)
        s = e.store_state()
        assert_states_equal(s, o.state(), Gh, Ph, Lh, "forged flags by reference")
        assert (s["terms_sorted"] == 0).sum() > 0


@pytest.mark.parametrize("mk", BACKENDS)
def test_start_and_install_rules(mk):
    """Start clears the proof when the last term exceeds currentTerm (not a
    reachable leader, but a valid engine state); an InstallSnapshot that
    replaces the log sets it."""
    st = _state()
    _set_log(st, 0, [0, 1, 4])                # leader, term 3 < last term 4
    _set_log(st, 3, [0, 1, 2])                # leader, normal
    _set_log(st, 7, [0, 3, 1])                # follower, not sorted
    e = mk(st)
    idx, term, isl, err = e.start(np.array([0, 3], np.int32))
    assert not err.any() and isl.all()
    s = _store(e)
    assert s["terms_sorted"][0] == 0 and s["terms_sorted"][3] == 1
    assert s["terms_sorted"][7] == 0
    from multiraft_amd._abi import IS_ARGS
    a = np.zeros(1, dtype=IS_ARGS)
    a["slot"], a["term"], a["leader_id"], a["last_included_index"], a["last_included_term"] = 7, 3, 0, 9, 2
    rep, fl, err = e.handle_install_snapshot(a)
    assert not err.any() and fl[0] == 32
    s = _store(e)
    assert s["terms_sorted"][7] == 1 and s["last_index"][7] == 9 and s["dummy_index"][7] == 9
    assert_terms_sorted_sound(s, G, P, L, "start / install")


@pytest.mark.parametrize("mk", BACKENDS)
def test_restore_and_load_compute_the_proof(mk):
    """mraft_restore and mraft_load_state compute the proof from the terms,
    whatever the source image claims."""
    st = _state()
    _set_log(st, 1, [0, 2, 1])
    _set_log(st, 2, [7, 1, 2])                # the dummy's term does not count
    st["terms_sorted"][:] = 1                  # a false claim, ignored on load
    e = mk(st)
    s = _store(e)
    assert s["terms_sorted"][1] == 0 and s["terms_sorted"][2] == 1
    assert np.array_equal(s["terms_sorted"], terms_sorted_exact(s, G, P, L))
    hdr, terms = e.read_persistent(np.array([1, 2], np.int32))
    hdr["slot"] = [4, 5]
    assert not e.restore(hdr, terms).any()
    s = _store(e)
    assert s["terms_sorted"][4] == 0 and s["terms_sorted"][5] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["tick", "fold"])
def test_withheld_proof_same_decisions_gpu(what):
    """The proof only skips reads: with terms_sorted all 0 (bound as is,
    mraft_bind_state) the tick and the reply fold run Go's downward scans and
    reach the same decisions and state as with the proof (config #3's mix,
    where a quarter of the groups have no entry of the current term)."""
    import torch

    from multiraft_amd import DEVICE
    Gs, Ps, Ls = 2048, 5, 512
    st, lp, _ = synth_tick_state(Gs, Ps, Ls, seed=synth_seed(3))
    assert st["terms_sorted"].all()
    dev = torch.device("cuda", 0)
    outs = []
    for proof in (1, 0):
        d = {k: torch.from_numpy(v.copy()).to(dev) for k, v in st.items()}
        d["terms_sorted"].fill_(proof)
        with Engine(Gs, Ps, Ls, alloc=False) as e:
            e.bind(d)
            if what == "tick":
                gf = torch.zeros(Gs, dtype=torch.int32, device=dev)
                e.replicate_tick(torch.from_numpy(lp).to(dev), gf, where=DEVICE)
                e.synchronize()
                res = gf.cpu().numpy()
            else:
                items, seg = synth_fold_batch(st, Gs, Ps, Ls, lp, seed=7)
                res = e.process_append_replies(items, seg)[0]
            outs.append((res, {k: v.cpu().numpy() for k, v in d.items()}))
    (r1, s1), (r0, s0) = outs
    assert np.array_equal(r1, r0)
    s1.pop("terms_sorted")
    s0.pop("terms_sorted")
    assert_states_equal(s1, s0, Gs, Ps, Ls, f"{what} with and without the proof")
    o = Oracle(Gs, Ps, Ls, st)
    if what == "tick":
        assert np.array_equal(r1, o.replicate_tick(lp))
    else:
        items, seg = synth_fold_batch(st, Gs, Ps, Ls, lp, seed=7)
        assert np.array_equal(r1, o.process_append_replies(items, seg)[0])
    assert_states_equal(s1, o.state(), Gs, Ps, Ls, f"{what} vs oracle")


def _history(mk, monotone, seed, steps=6):
    """Random sequences of every call that touches the logs — the fused tick,
    the message path by reference and by value (entries with their args'
    flag), Start, Snapshot, the InstallSnapshot exchange, restarts — on
    adversarial states (non-monotone terms unless `monotone`). Returns the
    backend and the states after each step."""
    from message_cases import all_follower_items, external_entries, results_of
    from random_states import random_tick_state
    from snapshot_cases import run_snapshot_scenario
    rng = np.random.default_rng(seed)
    Gh, Ph, Lh = 96, 5, 64
    st, lp = random_tick_state(rng, Gh, Ph, Lh, monotone=monotone)
    e = mk(Gh, Ph, Lh, st)
    seen = []
    for k in range(steps):
        op = k % 6
        if op == 0:
            e.replicate_tick(lp)
        elif op in (1, 2):
            lpv = np.where((lp >= 0) & (lp < Ph), lp, -1).astype(np.int32)
            slots, peers = all_follower_items(lpv, Gh, Ph)
            args, gerr = e.gather_append_args(slots, peers)
            ok = gerr == 0
            if op == 1:
                rep, herr = e.handle_append_entries(args[ok], None)
            else:
                a2, buf = external_entries(args[ok], np.ones(int(ok.sum()), bool), e.store_state(), Lh)
                rep, herr = e.handle_append_entries(a2, buf)
            res, seg = results_of(slots[ok], peers[ok], args[ok], rep, herr, Gh, Ph)
            e.process_append_replies(res, seg)
        elif op == 3:
            ld = np.array([g * Ph + lp[g] for g in range(Gh) if 0 <= lp[g] < Ph], np.int32)
            e.start(ld, rng.integers(1, 4, size=len(ld)).astype(np.int32))
        elif op == 4:
            run_snapshot_scenario(e, e.store_state(), Gh, Ph, Lh, np.where(lp < Ph, lp, -1), seed + k)
        else:
            sl = rng.choice(Gh * Ph, size=Gh // 4, replace=False).astype(np.int32)
            hdr, terms = e.read_persistent(sl)
            e.restore(hdr, terms)
        s = e.store_state()
        assert_terms_sorted_sound(s, Gh, Ph, Lh, f"step {k}")
        seen.append(s)
    return e, seen, (Gh, Ph, Lh)


@pytest.mark.parametrize("monotone", [True, False])
@pytest.mark.parametrize("seed", [11, 12])
def test_history_oracle(monotone, seed):
    """Every call keeps the proof sound on the oracle; on monotone states most
    replicas keep it."""
    e, seen, (Gh, Ph, Lh) = _history(lambda G_, P_, L_, st: Oracle(G_, P_, L_, st), monotone, seed)
    if monotone:
        assert seen[-1]["terms_sorted"].mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("monotone", [True, False])
@pytest.mark.parametrize("seed", [11, 12])
def test_history_gpu_equals_oracle(monotone, seed):
    """The same histories on libmraft_hip.so: identical state after every
    step, the proof included."""
    def gpu(G_, P_, L_, st):
        e = Engine(G_, P_, L_)
        e.load_state(st)
        return e
    _, so, dims = _history(lambda G_, P_, L_, st: Oracle(G_, P_, L_, st), monotone, seed)
    eg, sg, _ = _history(gpu, monotone, seed)
    for k, (a, b) in enumerate(zip(sg, so)):
        assert_states_equal(a, b, *dims, f"history step {k}")
    eg.close()
