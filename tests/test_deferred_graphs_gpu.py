"""Deferred items on the GPU: batches by reference whose
rows are read and written in random functional graphs — trees and chains
feeding cycles, cycles longer than the fallback's walk, self-references —
through mraft_handle_append_entries at the default stage, a stage too small
(64 words) and none (the fallback: chains hand-off, short cycles on one wave
each, the rest on the last workgroup), each twice on one engine: the first
call on the minimal deferred grid (no earlier count: 512 workgroups, and 8
through MRAFT_DEFER_GRID_MIN), the second on the grid the first call's count
asked for. GPU == oracle (which copies every item's
entries before the call, as the reference's gather does,
src/raft/raft_append_entry.go:50-54) on replies, errors and state."""
import numpy as np
import pytest

from message_cases import deferred_graph_batch, deferred_graph_state
from oracle_lib import Oracle, assert_states_equal

from multiraft_amd import Engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gmin", [None, 8])
@pytest.mark.parametrize("cap", [None, 64, 0])
@pytest.mark.parametrize("shape", ["random", "long_cycle", "dense"])
def test_deferred_graphs_gpu(shape, cap, gmin, monkeypatch):
    # gmin 8: the deferred launch's minimum grid far below the item count
    # (MRAFT_DEFER_GRID_MIN, read at mraft_create): the grid-stride loops and,
    # in the fallback, workgroups without a cycle buffer
    if gmin is not None:
        monkeypatch.setenv("MRAFT_DEFER_GRID_MIN", str(gmin))
    G, P, L = 64, 5, 64
    rng = np.random.default_rng({"random": 700, "long_cycle": 701, "dense": 702}[shape])
    st, c = deferred_graph_state(G, P, L, rng)
    n_items = {"random": 200, "long_cycle": 220, "dense": G * P}[shape]
    a = deferred_graph_batch(st, G, P, L, c, rng, n_items,
                             long_cycle=40 if shape == "long_cycle" else 0,
                             self_refs=3 if shape != "random" else 0)
    o = Oracle(G, P, L, st)
    orep, oerr = o.handle_append_entries(a, None)
    want = o.state()
    assert (oerr == 0).sum() > n_items // 2
    with Engine(G, P, L) as e:
        if cap is not None:
            e.set_stage_capacity(cap)
        for call in range(2):
            e.load_state(st)
            rep, err = e.handle_append_entries(a, None)
            assert np.array_equal(err, oerr), f"call {call}: errors"
            assert np.array_equal(rep, orep), f"call {call}: replies"
            assert_states_equal(e.store_state(), want, G, P, L, f"{shape}, stage {cap}, call {call}")


def test_deferred_then_plain_gpu():
    """A deferred-heavy batch, then a batch with no deferred item (the grid
    falls back to the minimum), then the heavy one again: every call exact."""
    from message_cases import all_follower_items
    from multiraft_amd import synth_tick_state
    G, P, L = 64, 5, 64
    rng = np.random.default_rng(703)
    st, c = deferred_graph_state(G, P, L, rng)
    heavy = deferred_graph_batch(st, G, P, L, c, rng, G * P)
    st2, lp, _ = synth_tick_state(G, P, L, seed=704)
    with Engine(G, P, L) as e:
        for k, (state, batch) in enumerate([(st, heavy), (st2, None), (st, heavy)]):
            o = Oracle(G, P, L, state)
            e.load_state(state)
            if batch is None:
                slots, peers = all_follower_items(lp, G, P)
                batch, gerr = e.gather_append_args(slots, peers)
                batch = batch[gerr == 0]
            rep, err = e.handle_append_entries(batch, None)
            orep, oerr = o.handle_append_entries(batch, None)
            assert np.array_equal(err, oerr) and np.array_equal(rep, orep), k
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"call {k}")
