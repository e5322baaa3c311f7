"""Randomised parity of the election storm (StartElection ->
HandleRequestVote x voters -> tally, src/raft/raft_election.go:4-77 with
isLogUpToDate raft_log.go:99-104) against the C oracle: seeded config-#5
states with every group size P = 1..8, storms of 1-96 rounds, timeout masks
from the generator or drawn at random densities (sparse to every replica at
once), leaders already in place, rings started at random heads (the voters'
last terms read through the wrap), and two launches back to back on one
state — group flags and the whole state equal after each."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal, rotate_rings

from multiraft_amd import Engine, synth_election_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", list(range(32)))
def test_election_storm_fuzz_gpu(seed):
    rng = np.random.default_rng(9100 + seed)
    P = 1 + seed % 8
    G = int(rng.integers(100, 1500))
    L = int(rng.choice([8, 13, 16, 64]))
    R = int(rng.integers(1, 97))
    st, mask = synth_election_state(G, P, L, seed=9300 + seed, rounds=R)
    if seed % 3 == 1:
        dens = float(rng.choice([0.02, 0.3, 0.9, 1.0]))
        bits = (rng.random((R, G, P)) < dens).astype(np.uint8)
        mask = (bits << np.arange(P, dtype=np.uint8)).sum(axis=2).astype(np.uint8)
    if seed % 2 == 0:
        st = rotate_rings(st, G, P, L, rng, frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        for launch in range(2):
            gf = e.election_rounds(mask)
            assert np.array_equal(gf, o.election_rounds(mask)), (seed, launch)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"seed {seed}, launch {launch}")
