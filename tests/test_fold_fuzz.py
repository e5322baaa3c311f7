"""Randomised parity of the reply fold (processAppendEntriesReply + a1,
src/raft/raft_append_entry.go:66-105) against the C oracle: seeded states
whose logs do and do not keep their terms in order (the terms_sorted proof
settles an a1 range by its top term only where it holds, include/mraft.h),
rings started at random heads, and reply segments of up to 8, 40 or 150
replies (the lane-group fold, the long-segment path and the pending a1 scans,
each grid-striding over its device list), on engines that fold twice in a row
— flags, item errors and the whole state equal after each call."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal, random_reply_segments, rotate_rings
from random_states import random_tick_state

from multiraft_amd import Engine, synth_tick_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", list(range(24)))
def test_fold_fuzz_gpu(seed):
    rng = np.random.default_rng(5600 + seed)
    P = int(rng.choice([2, 3, 5, 7, 8]))
    max_len = int(rng.choice([8, 40, 150]))
    if seed % 2:
        G, L = int(rng.integers(64, 400)), int(rng.choice([64, 65, 128]))
        st, lp = random_tick_state(rng, G, P, L, monotone=bool(rng.random() < 0.5))
    else:
        G, L = int(rng.choice([256, 1024])), int(rng.choice([128, 131, 512]))
        st, lp, _ = synth_tick_state(G, P, L, seed=5700 + seed)
    if rng.random() < 0.6:
        st = rotate_rings(st, G, P, L, rng, frac=0.8)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        for call in range(2):
            items, seg = random_reply_segments(o.state(), G, P, lp, seed=5800 + 10 * seed + call, max_len=max_len)
            f, err = e.process_append_replies(items, seg)
            of, oerr = o.process_append_replies(items, seg)
            assert np.array_equal(err, oerr) and np.array_equal(f, of), (seed, call)
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"seed {seed}, call {call}")
