"""The log ring (include/mraft.h: Index i at row[(log_head + i - dummy) mod L]).

Every state is run twice: as generated (every head at 0) and with each
replica's ring rotated to a random head (the same logical state). On the CPU
the oracle must give the same decisions and the same logs in Index order
either way; Snapshot and InstallSnapshot's sliceFrom (raft_snapshot.go:10,40)
must move no term. On the GPU every entry point must match the oracle bit for
bit on rotated states, ring positions included (the wrap inside the streaming
pass, the scans, appends, persistence read-out and by-reference entries)."""
import numpy as np
import pytest

from message_cases import all_follower_items, external_entries, results_of
from oracle_lib import Oracle, assert_states_equal, logical_logs, rotate_rings
from random_states import random_tick_state

from multiraft_amd import Engine, synth_seed, synth_tick_state


def _rot(st, G, P, L, seed, frac=1.0):
    return rotate_rings(st, G, P, L, np.random.default_rng(seed), frac)


# ---------------------------------------------------------------- CPU (oracle)

@pytest.mark.parametrize("P,L,snap", [(3, 16, False), (5, 64, True), (5, 256, False), (7, 40, True)])
def test_oracle_tick_is_rotation_invariant(P, L, snap):
    G = 300
    rng = np.random.default_rng(900 + P + L)
    st, lp = random_tick_state(rng, G, P, L, snap=snap)
    rt = _rot(st, G, P, L, 5)
    a, b = Oracle(G, P, L, st), Oracle(G, P, L, rt)
    assert a.replicate_tick_count(lp) == b.replicate_tick_count(lp)
    assert np.array_equal(a.replicate_tick(lp), b.replicate_tick(lp))
    assert_states_equal(a.state(), b.state(), G, P, L, "rotated tick", heads=False)


def test_oracle_snapshot_moves_no_term():
    G, P, L = 64, 5, 32
    st, lp, _ = synth_tick_state(G, P, L, seed=31)
    rt = _rot(st, G, P, L, 6)
    o = Oracle(G, P, L, rt)
    slots = np.arange(G * P, dtype=np.int32)
    idx = np.minimum(rt["dummy_index"] + 3, rt["last_index"]).astype(np.int32)
    before = o.state()
    assert (o.snapshot(slots, idx) == 0).all()
    after = o.state()
    assert np.array_equal(after["log_term"], before["log_term"])           # O(1): no term moved
    assert np.array_equal(after["dummy_index"], np.maximum(idx, before["dummy_index"]))
    moved = after["dummy_index"] - before["dummy_index"]
    assert np.array_equal(after["log_head"], (before["log_head"] + moved) % L)
    # the logs in Index order are the old ones from the new dummy on
    la, lb = logical_logs(after, G, P, L), logical_logs(before, G, P, L)
    for r in range(0, G * P, 37):
        k = int(after["last_index"][r] - after["dummy_index"][r]) + 1
        assert np.array_equal(la[r, :k], lb[r, moved[r]:moved[r] + k])


def test_oracle_by_reference_entries_across_the_wrap():
    """Entries by reference whose range wraps around the leader's ring equal
    the same entries delivered in a contiguous buffer."""
    G, P, L = 128, 5, 64
    st, lp, _ = synth_tick_state(G, P, L, seed=44)
    rt = _rot(st, G, P, L, 7)
    slots, peers = all_follower_items(lp, G, P)
    a, b = Oracle(G, P, L, rt), Oracle(G, P, L, rt)
    args, gerr = a.gather_append_args(slots, peers)
    b.gather_append_args(slots, peers)
    ok = gerr == 0
    rep, herr = a.handle_append_entries(args, None)
    a2, buf = external_entries(args, ok, rt, L)   # the ring unrolled through log_head
    rep2, herr2 = b.handle_append_entries(a2[ok], buf)
    assert np.array_equal(rep[ok], rep2) and np.array_equal(herr[ok], herr2)
    assert_states_equal(a.state(), b.state(), G, P, L, "by reference across the wrap")
    # some ranges did wrap
    h = rt["log_head"][slots[ok]]
    k0 = args["entries_offset"][ok] % L
    assert ((h + k0) % L + args["n_entries"][ok] > L).any()


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("P,L,snap,mono", [(2, 8, False, False), (3, 16, True, False), (5, 12, False, False),
                                           (5, 256, True, False), (5, 1024, False, True), (8, 40, True, False),
                                           (7, 64, False, False)])
def test_tick_rotated_gpu(P, L, snap, mono):
    G = 700
    rng = np.random.default_rng(3100 + P * 100 + L)
    st, lp = random_tick_state(rng, G, P, L, monotone=mono, snap=snap)
    rt = _rot(st, G, P, L, 8, frac=0.8)
    o = Oracle(G, P, L, rt)
    with Engine(G, P, L) as e:
        e.load_state(rt)
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        gf = e.replicate_tick(lp)
        assert np.array_equal(gf, o.replicate_tick(lp))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "rotated tick")


@pytest.mark.gpu
def test_tick_config3_shape_rotated_gpu():
    """Config-#3 generator at full L (4,096), rings rotated: the dwordx4
    streaming pass wraps inside chunks; two ticks."""
    G, P, L = 2048, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    rt = _rot(st, G, P, L, 9)
    o = Oracle(G, P, L, rt)
    with Engine(G, P, L) as e:
        e.load_state(rt)
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        for k in range(2):
            assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp, nthreads=8)), k
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"rotated config-3 tick {k}")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["reference", "aligned", "misaligned"])
def test_message_path_rotated_gpu(mode):
    G, P, L = 256, 5, 512
    st, lp, _ = synth_tick_state(G, P, L, seed=55)
    rt = _rot(st, G, P, L, 10)
    slots, peers = all_follower_items(lp, G, P)
    o = Oracle(G, P, L, rt)
    with Engine(G, P, L) as e:
        e.load_state(rt)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr)
        ok = gerr == 0
        if mode == "reference":
            rep, herr = e.handle_append_entries(args, None)
            orep, oherr = o.handle_append_entries(args, None)
        else:
            a2, buf = external_entries(args, ok, rt, L, misalign=(mode == "misaligned"))
            args, slots, peers = args[ok], slots[ok], peers[ok]
            rep, herr = e.handle_append_entries(a2[ok], buf)
            orep, oherr = o.handle_append_entries(a2[ok], buf)
        assert np.array_equal(herr, oherr) and np.array_equal(rep, orep)
        res, seg = results_of(slots, peers, args, rep, herr, G, P)
        f, ferr = e.process_append_replies(res, seg)
        of, oferr = o.process_append_replies(res, seg)
        assert np.array_equal(f, of) and np.array_equal(ferr, oferr)
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"rotated message path ({mode})")


@pytest.mark.gpu
@pytest.mark.parametrize("P,L", [(3, 16), (5, 40), (7, 32), (3, 13), (5, 37), (7, 99)])
def test_snapshot_and_persistence_rotated_gpu(P, L):
    """Snapshot / InstallSnapshot as ring rebases, then persistence read-out
    (in Index order across the wrap), restore (head back to 0) and Start; at
    capacities that are and are not a multiple of four."""
    from snapshot_cases import run_snapshot_scenario
    G = 300
    rng = np.random.default_rng(4100 + P + L)
    st, lp = random_tick_state(rng, G, P, L)
    lp = np.where((lp >= 0) & (lp < P), lp, 0).astype(np.int32)
    rt = _rot(st, G, P, L, 11)
    o = Oracle(G, P, L, rt)
    with Engine(G, P, L) as e:
        e.load_state(rt)
        go = run_snapshot_scenario(e, rt, G, P, L, lp, seed=12)
        oo = run_snapshot_scenario(o, rt, G, P, L, lp, seed=12)
        for k in oo:
            assert np.array_equal(go[k], oo[k]), k
        assert_states_equal(e.store_state(), o.state(), G, P, L, "rotated snapshot scenario")
        slots = np.arange(0, G * P, 3, dtype=np.int32)
        hdr, terms = e.read_persistent(slots)
        ohdr, oterms = o.read_persistent(slots)
        assert np.array_equal(hdr, ohdr) and np.array_equal(terms, oterms)
        assert np.array_equal(e.restore(hdr, terms), o.restore(hdr, terms))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "rotated restore")
        ss = rng.integers(0, G * P, 120).astype(np.int32)
        cnt = rng.integers(1, 6, 120).astype(np.int32)
        for a, b in zip(e.start(ss, cnt), o.start(ss, cnt)):
            assert np.array_equal(a, b)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "rotated start")


@pytest.mark.gpu
def test_elections_rotated_gpu():
    from multiraft_amd import synth_election_state
    G, P, L = 1024, 7, 8
    st, mask = synth_election_state(G, P, L, seed=77, rounds=16)
    rt = _rot(st, G, P, L, 13)
    o = Oracle(G, P, L, rt)
    with Engine(G, P, L) as e:
        e.load_state(rt)
        assert np.array_equal(e.election_rounds(mask), o.election_rounds(mask))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "rotated election rounds")
