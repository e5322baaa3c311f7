"""Randomised multi-step parity of the fused replication tick
(appendOneRound -> HandleAppendEntries -> processAppendEntriesReply ->
advanceCommitIndexForLeader, src/raft/raft_append_entry.go:20-162, with the
InstallSnapshot branch :27-34 and raft_snapshot.go:15-69) against the C
oracle: seeded random states (tests/random_states.py: diverging follower
tails, snapshot-heavy variants, monotone and non-monotone term sequences,
bad-state leaders), rings started at random heads, the tick as 1, 2 or 3
engine-owned shards, log capacities with and without L % 4 == 0 (the
passes' dwordx4 and dword forms), and between ticks Start() on random leaders
(raft.go:90-104) and leader changes — four ticks per case, every group flag
and the whole state equal to the oracle's after each."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal, rotate_rings
from random_states import random_tick_state

from multiraft_amd import Engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", list(range(48)))
def test_tick_multistep_fuzz_gpu(seed):
    rng = np.random.default_rng(7700 + seed)
    P = int(rng.choice([2, 3, 5, 7, 8]))
    L = int(rng.choice([32, 37, 64, 99, 128, 256]))
    G = int(rng.integers(150, 500))
    st, lp = random_tick_state(rng, G, P, L, monotone=bool(rng.random() < 0.5), snap=bool(rng.random() < 0.3))
    if rng.random() < 0.7:
        st = rotate_rings(st, G, P, L, rng, frac=float(rng.uniform(0.3, 1.0)))
    shards = int(rng.choice([1, 2, 3]))
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.set_tick_shards(min(shards, G))
        for step in range(4):
            gf = e.replicate_tick(lp)
            ogf = o.replicate_tick(lp)
            assert np.array_equal(gf, ogf), (seed, step)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"seed {seed}, step {step}, shards {shards}")
            # Start() on a random subset of groups' current leader peers (a
            # non-leader answers isLeader = false), 0-3 commands each
            g = rng.choice(G, size=max(1, G // 5), replace=False)
            slots = (g * P + lp[g]).astype(np.int32)
            counts = rng.integers(0, 4, size=len(slots)).astype(np.int32)
            got = e.start(slots, counts)
            want = o.start(slots, counts)
            for a, b in zip(got, want):
                assert np.array_equal(a, b), (seed, step, "start")
            # a few groups tick another peer next (a stale or non-leader view)
            moved = rng.random(G) < 0.1
            lp = np.where(moved, rng.integers(0, P, size=G), lp).astype(np.int32)
