"""Randomised parity of the message-level AppendEntries handler
(HandleAppendEntries, src/raft/raft_append_entry.go:108-162, matchLog
raft_log.go:92-96) against the C oracle: seeded batches that mix what the
handler's classification must keep apart, on states whose rings start at
random heads (so the pass meets leader and follower rows aligned alike and
not: its dwordx4 and dword forms, include/mraft.h log layout):

* by reference: gathered follower items, stale second leaders and rings of
  2..P stale leaders (deferred, staged and ordered items), shuffled (sets cut
  at random), with duplicates of receiving slots (MRAFT_ITEM_DUP_SLOT) and
  MRAFT_AE_ENTRIES_SORTED flags set where they do not hold; stage capacity
  0, small or default;
* by value: the same items' entries copied into a caller buffer at
  misaligned positions.

Group sizes P = 2..8 (one to seven messages per set) and log capacities with
and without L % 4 == 0. Each case: replies, item errors and the whole state
equal the oracle's."""
import numpy as np
import pytest

from message_cases import all_follower_items, external_entries, stale_cycle_state, stale_second_leader_state
from oracle_lib import Oracle, assert_states_equal, rotate_rings

from multiraft_amd import Engine, synth_tick_state
from multiraft_amd._abi import AE_ENTRIES_SORTED

pytestmark = pytest.mark.gpu

SEEDS = list(range(40))


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    G = int(rng.choice([64, 128, 192]))
    P = int(rng.choice([2, 3, 5, 7, 8]))
    L = int(rng.choice([64, 77, 128, 141, 256]))
    st, lp, _ = synth_tick_state(G, P, L, seed=4242 + seed)
    kind = seed % 3
    if kind == 0:
        slots, peers = all_follower_items(lp, G, P)
    elif kind == 1:
        st, slots, peers = stale_second_leader_state(st, lp, G, P, L, rng, range(0, G, 3))
    else:
        k = int(rng.integers(2, P + 1))
        st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(1, G, 4), k)
    if seed % 2 == 0:
        st = rotate_rings(st, G, P, L, rng, frac=0.7)
    return rng, G, P, L, st, slots, peers


def _perturb(rng, args, P, G):
    """Shuffle some runs (cuts sets), duplicate some receiving slots, and set
    the sorted-entries flag on random items whether or not it holds."""
    b = args.copy()
    n = len(b)
    if n > 4:
        cut = rng.choice(n, size=max(1, n // 8), replace=False)
        b[np.sort(cut)] = b[cut]                                   # a scattered permutation
        dups = rng.choice(n, size=max(1, n // 16), replace=False)
        src = rng.choice(n, size=len(dups))
        b["slot"][dups] = b["slot"][src]                          # two items for one replica slot
    fl = rng.random(n) < 0.3
    b["flags"][fl] |= AE_ENTRIES_SORTED
    return b


@pytest.mark.parametrize("seed", SEEDS)
def test_handler_by_reference_fuzz_gpu(seed):
    rng, G, P, L, st, slots, peers = _case(seed)
    cap = [0, 64, None][seed % 3]
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap is not None:
            e.set_stage_capacity(cap)
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr), seed
        batch = _perturb(rng, args[gerr == 0], P, G)
        rep, herr = e.handle_append_entries(batch, None)
        orep, oherr = o.handle_append_entries(batch, None)
        assert np.array_equal(herr, oherr), seed
        assert np.array_equal(rep, orep), seed
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"seed {seed}, stage {cap}")


@pytest.mark.parametrize("seed", SEEDS[:16])
def test_handler_by_value_fuzz_gpu(seed):
    rng, G, P, L, st, slots, peers = _case(seed)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        args, gerr = e.gather_append_args(slots, peers)
        ok = gerr == 0
        ext, buf = external_entries(args, ok, st, L, misalign=True)
        batch = _perturb(rng, ext[ok], P, G)
        rep, herr = e.handle_append_entries(batch, buf)
        o.gather_append_args(slots, peers)
        orep, oherr = o.handle_append_entries(batch, buf)
        assert np.array_equal(herr, oherr), seed
        assert np.array_equal(rep, orep), seed
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"seed {seed}, by value")
