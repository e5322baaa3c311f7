"""Log capacities L that are not a multiple of four. Every other parity suite
runs at L = 4k, where the leader's and a follower's rings wrap at a dwordx4
boundary and the streaming passes take their dwordx4 forms; at L % 4 != 0 the
tick and the by-reference handler take the dword forms (mraft_pass.h
pass_chunk<1, false> and the copy loop's dword form) and every ring wrap falls
inside a vector's span. Seeded random states (diverging tails, snapshots,
non-monotone terms), rings started at random heads, against the C oracle:

* the fused tick, 1 or 2 shards, three ticks with Start() between them;
* the message path gather -> handle -> fold, entries by reference and by
  value, with and without stale second leaders (deferred and staged items);
* rings of stale leaders at stage capacities 0 / 64 / default (the ordered
  fallback and its cycle buffer included);
* the election storm, the voters' last terms read through the wrap;
* the smallest engines (G, P, L down to 1, 1, 1);
* L = 4k with the log bound 4 B past a 16-B boundary (mraft_bind_state): the
  same dword forms, chosen by the base address instead of the capacity."""
import numpy as np
import pytest

from message_cases import (all_follower_items, external_entries, results_of, stale_cycle_state,
                           stale_second_leader_state)
from oracle_lib import Oracle, assert_states_equal, rotate_rings, terms_sorted_exact
from random_states import random_tick_state

from multiraft_amd import Engine, synth_election_state, synth_tick_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [5, 9, 13, 37, 50, 99, 130, 1023])
def test_tick_odd_capacity_gpu(L):
    rng = np.random.default_rng(8800 + L)
    for P, shards in ((3, 1), (5, 2), (7, 2)):
        G = 240
        st, lp = random_tick_state(rng, G, P, L, monotone=bool(L % 2), snap=(L % 3 == 0))
        st = rotate_rings(st, G, P, L, rng, frac=0.8)
        o = Oracle(G, P, L, st)
        with Engine(G, P, L) as e:
            e.load_state(st)
            e.set_tick_shards(shards)
            for step in range(3):
                gf = e.replicate_tick(lp)
                assert np.array_equal(gf, o.replicate_tick(lp)), (L, P, step)
                assert_states_equal(e.store_state(), o.state(), G, P, L, f"L {L}, P {P}, step {step}")
                g = rng.choice(G, size=G // 4, replace=False)
                slots = (g * P + np.clip(lp[g], 0, P - 1)).astype(np.int32)
                counts = rng.integers(1, 4, size=len(slots)).astype(np.int32)
                for a, b in zip(e.start(slots, counts), o.start(slots, counts)):
                    assert np.array_equal(a, b), (L, P, step, "start")


@pytest.mark.parametrize("L", [13, 37, 99, 130])
@pytest.mark.parametrize("stale", [False, True])
@pytest.mark.parametrize("by", ["reference", "value"])
def test_message_path_odd_capacity_gpu(L, stale, by):
    rng = np.random.default_rng(9900 + L + 7 * stale + 3 * (by == "value"))
    G, P = 192, 5
    st, lp, _ = synth_tick_state(G, P, L, seed=4400 + L)
    if stale:
        st, slots, peers = stale_second_leader_state(st, lp, G, P, L, rng, range(0, G, 3))
    else:
        slots, peers = all_follower_items(lp, G, P)
    st = rotate_rings(st, G, P, L, rng, frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        for step in range(2):
            args, gerr = e.gather_append_args(slots, peers)
            oargs, ogerr = o.gather_append_args(slots, peers)
            assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr), (L, step)
            ok = gerr == 0
            if by == "value":
                ext, buf = external_entries(args, ok, o.state(), L, misalign=True)
                batch = ext[ok]
            else:
                batch, buf = args[ok], None
            rep, herr = e.handle_append_entries(batch, buf)
            orep, oherr = o.handle_append_entries(batch, buf)
            assert np.array_equal(herr, oherr) and np.array_equal(rep, orep), (L, step)
            res, seg = results_of(slots[ok], peers[ok], args[ok], rep, herr, G, P)
            f, ferr = e.process_append_replies(res, seg)
            of, oferr = o.process_append_replies(res, seg)
            assert np.array_equal(f, of) and np.array_equal(ferr, oferr), (L, step)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"L {L}, {by}, stale {stale}, step {step}")


@pytest.mark.parametrize("L", [13, 37, 99])
@pytest.mark.parametrize("cap", [0, 64, None])
def test_stale_rings_odd_capacity_gpu(L, cap):
    """Rings of 2..P stale leaders sending to each other: every item deferred,
    its entries staged (capacity 64 words or the default) or, with no stage,
    run in order with each cycle broken through the L-word cycle buffer."""
    rng = np.random.default_rng(7300 + L + (cap or 1))
    G, P = 160, 5
    st, lp, _ = synth_tick_state(G, P, L, seed=7400 + L)
    st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(1, G, 4), int(rng.integers(2, P + 1)))
    st = rotate_rings(st, G, P, L, rng, frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap is not None:
            e.set_stage_capacity(cap)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr), L
        ok = gerr == 0
        rep, herr = e.handle_append_entries(args[ok], None)
        orep, oherr = o.handle_append_entries(args[ok], None)
        assert np.array_equal(herr, oherr) and np.array_equal(rep, orep), (L, cap)
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"L {L}, stage {cap}")


@pytest.mark.parametrize("L", [5, 13, 37])
def test_election_storm_odd_capacity_gpu(L):
    G, P, R = 1000, 5, 24
    st, mask = synth_election_state(G, P, L, seed=9500 + L, rounds=R)
    st = rotate_rings(st, G, P, L, np.random.default_rng(L), frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        for launch in range(2):
            assert np.array_equal(e.election_rounds(mask), o.election_rounds(mask)), (L, launch)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"L {L}, launch {launch}")


@pytest.mark.parametrize("off", [1, 2, 3])
def test_misaligned_log_base_gpu(off):
    """A caller-bound state whose log_term starts `off` words past a 16-B
    boundary: the tick and the by-reference handler cannot use dwordx4 loads
    on it and take the dword forms; two ticks, then a message step."""
    import torch
    from multiraft_amd._abi import DEVICE  # noqa: F401  (device-bound state)
    rng = np.random.default_rng(6100 + off)
    G, P, L = 256, 5, 64
    st, lp = random_tick_state(rng, G, P, L, monotone=True)
    st = rotate_rings(st, G, P, L, rng, frac=0.8)
    st["terms_sorted"] = terms_sorted_exact(st, G, P, L).astype(np.int32)  # bind takes the proof as given
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(v.copy()).to(dev) for k, v in st.items()}
    big = torch.zeros(len(st["log_term"]) + 4, dtype=torch.int32, device=dev)
    big[off:off + len(st["log_term"])] = d["log_term"]
    d["log_term"] = big[off:off + len(st["log_term"])]
    assert d["log_term"].data_ptr() % 16 == 4 * off
    o = Oracle(G, P, L, st)
    with Engine(G, P, L, alloc=False) as e:
        e.bind(d)
        for step in range(2):
            gf = e.replicate_tick(lp)
            assert np.array_equal(gf, o.replicate_tick(lp)), (off, step)
        slots, peers = all_follower_items(np.clip(lp, 0, P - 1), G, P)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr), off
        ok = gerr == 0
        rep, herr = e.handle_append_entries(args[ok], None)
        orep, oherr = o.handle_append_entries(args[ok], None)
        assert np.array_equal(herr, oherr) and np.array_equal(rep, orep), off
        e.synchronize()
    got = {k: v.cpu().numpy() for k, v in d.items()}
    assert_states_equal(got, o.state(), G, P, L, f"log base +{off} words")


@pytest.mark.parametrize("G,P,L", [(1, 1, 1), (1, 2, 1), (2, 3, 2), (3, 8, 3), (1, 8, 4), (2, 5, 1), (5, 2, 2)])
def test_tiny_shapes_gpu(G, P, L):
    """The smallest engines: one group, one peer, a log holding only the dummy
    entry (every append overflows: MRAFT_ITEM_LOG_FULL), all eight peers on a
    three-entry ring. Three ticks with Start() between, then a message step."""
    rng = np.random.default_rng(100 + G * 10 + P + L)
    st, lp = random_tick_state(rng, G, P, L)
    st = rotate_rings(st, G, P, L, rng, frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        for step in range(3):
            assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp)), (G, P, L, step)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"{G}x{P}x{L}, step {step}")
            slots = (np.arange(G) * P + np.clip(lp, 0, P - 1)).astype(np.int32)
            for a, b in zip(e.start(slots, np.ones(G, np.int32)), o.start(slots, np.ones(G, np.int32))):
                assert np.array_equal(a, b), (G, P, L, step, "start")
        slots, peers = all_follower_items(np.clip(lp, 0, P - 1), G, P)
        if len(slots):
            args, gerr = e.gather_append_args(slots, peers)
            oargs, ogerr = o.gather_append_args(slots, peers)
            assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr)
            ok = gerr == 0
            rep, herr = e.handle_append_entries(args[ok], None)
            orep, oherr = o.handle_append_entries(args[ok], None)
            assert np.array_equal(herr, oherr) and np.array_equal(rep, orep)
            res, seg = results_of(slots[ok], peers[ok], args[ok], rep, herr, G, P)
            f, ferr = e.process_append_replies(res, seg)
            of, oferr = o.process_append_replies(res, seg)
            assert np.array_equal(f, of) and np.array_equal(ferr, oferr)
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{G}x{P}x{L}, message step")
