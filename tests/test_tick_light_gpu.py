"""The light tick (MRAFT_TICK_LIGHT, mraft_set_tick_mode in include/mraft.h):
one launch settles, eight Raft groups per wave, every group whose followers all
reply success without a compare (a heartbeat, or an append at the follower's
last Index) and whose commitIndex settles at log[last]; a second launch runs
every other group through the full tick. Both are the reference's
appendOneRound -> HandleAppendEntries -> processAppendEntriesReply ->
advanceCommitIndexForLeader (src/raft/raft_append_entry.go:20-162, with
Start, src/raft/raft.go:90-104, between ticks).

Every case compares the GPU with the CPU oracle bit for bit after every tick
(group flags, the fused GetState words where exported, the whole state and
its persist bits), and reads which path the groups took
(mraft_tick_light_fallbacks): steady-state runs where most groups settle in
the light launch, seeded random states where most do not, a batch past the
light launch's 64-entry span after a steady tick (its fallback grid, sized
from the previous count, is then far smaller than the list: the grid-stride
loop), the top of the Index domain, shards, P = 1 and the mode calls."""
import numpy as np
import pytest

from message_cases import shift_indices, top_offset
from oracle_lib import Oracle, assert_states_equal, rotate_rings
from random_states import random_tick_state

from multiraft_amd import TICK_AUTO, TICK_FULL, TICK_LIGHT, Engine, MraftError, synth_tick_state

pytestmark = pytest.mark.gpu


def _active(gf):
    return int((gf & 1).astype(bool).sum())


def _step(e, o, lp, G, P, L, ctx, export):
    if export:
        gf, c, tl = e.replicate_tick_export(lp)
    else:
        gf = e.replicate_tick(lp)
    ogf = o.replicate_tick(lp)
    assert np.array_equal(gf, ogf), f"{ctx}: group flags"
    if export:  # the GetState words after the tick
        oc, otl = o.export_group_status(lp)
        assert np.array_equal(c, oc) and np.array_equal(tl, otl), f"{ctx}: export words"
    assert_states_equal(e.store_state(), o.state(), G, P, L, ctx)
    return gf


def _start_all(e, o, lp, G, P, rng, cmax, frac=1.0):
    g = np.flatnonzero(rng.random(G) < frac)
    if len(g) == 0:
        return
    slots = (g * P + lp[g]).astype(np.int32)
    counts = rng.integers(0, cmax + 1, size=len(slots)).astype(np.int32)
    for a, b in zip(e.start(slots, counts), o.start(slots, counts)):
        assert np.array_equal(a, b), "start"


def _steady_run(G, P, L, seed, shards, steps, cmax=4, export=False, state=None, lp=None):
    rng = np.random.default_rng(seed)
    if state is None:
        state, lp, _ = synth_tick_state(G, P, L, seed=seed)
    o = Oracle(G, P, L, state)
    fbs = []
    with Engine(G, P, L) as e:
        e.load_state(state)
        e.set_tick_shards(min(shards, G))
        e.set_tick_mode(TICK_LIGHT)
        assert e.tick_mode() == TICK_LIGHT
        for k in range(steps):
            gf = _step(e, o, lp, G, P, L, f"seed {seed} step {k}", export)
            fbs.append((e.tick_light_fallbacks(), _active(gf)))
            _start_all(e, o, lp, G, P, rng, cmax)
    return fbs


@pytest.mark.parametrize("P,L,shards", [(3, 64, 1), (5, 256, 2), (8, 99, 1), (5, 128, 3), (2, 37, 1), (7, 512, 2)])
def test_light_steady_state_gpu(P, L, shards):
    """Ticks with Start() of 0-4 entries at every leader between them: after
    the first ticks have repaired the seeded conflicts, most groups settle in
    the light launch."""
    G = 1024
    fbs = _steady_run(G, P, L, 9100 + P * 7 + L, shards, steps=8, export=(shards == 2))
    fb, act = fbs[-1]
    assert 0 <= fb < act, fbs            # the light launch settled groups
    assert fb <= act // 2, fbs           # ... most of the active ones, once steady


@pytest.mark.parametrize("seed", list(range(16)))
def test_light_fuzz_gpu(seed):
    """Seeded random states (tests/random_states.py: diverging tails, snapshot
    branches, bad-state leaders, rotated rings), 1-3 shards, Start() and leader
    moves between ticks: every path of the full tick mixed with the light one."""
    rng = np.random.default_rng(8800 + seed)
    P = int(rng.choice([2, 3, 5, 7, 8]))
    L = int(rng.choice([32, 37, 64, 99, 128, 256]))
    G = int(rng.integers(150, 700))
    st, lp = random_tick_state(rng, G, P, L, monotone=bool(rng.random() < 0.5), snap=bool(rng.random() < 0.3))
    if rng.random() < 0.7:
        st = rotate_rings(st, G, P, L, rng, frac=float(rng.uniform(0.3, 1.0)))
    shards = int(rng.choice([1, 2, 3]))
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.set_tick_shards(min(shards, G))
        e.set_tick_mode(TICK_LIGHT)
        for step in range(6):
            _step(e, o, lp, G, P, L, f"seed {seed} step {step} shards {shards}", export=bool(step & 1))
            assert e.tick_light_fallbacks() >= 0
            _start_all(e, o, lp, G, P, rng, 3, frac=0.5)
            moved = rng.random(G) < 0.05
            lp = np.where(moved, rng.integers(0, P, size=G), lp).astype(np.int32)


def test_light_span_and_grid_stride_gpu():
    """Steady ticks (small fallback counts: the next fallback grid is
    max(2,048, twice the count) workgroups), then Start() of 70 entries at
    every leader: every group whose Start fits its ring exceeds the light
    launch's 64-entry span and goes to the full tick, more groups than the
    grid has workgroups (its grid-stride loop); then steady again."""
    G, P, L = 6000, 5, 512
    rng = np.random.default_rng(77)
    st, lp, _ = synth_tick_state(G, P, L, seed=4242)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.set_tick_mode(TICK_LIGHT)
        assert e.tick_light_fallbacks() == -1  # no light tick yet
        for k in range(5):
            _step(e, o, lp, G, P, L, f"steady {k}", False)
            _start_all(e, o, lp, G, P, rng, 2)
        fb0 = e.tick_light_fallbacks()
        g = np.arange(G)
        slots = (g * P + lp).astype(np.int32)
        counts = np.full(G, 70, np.int32)
        for a, b in zip(e.start(slots, counts), o.start(slots, counts)):
            assert np.array_equal(a, b)
        gf = _step(e, o, lp, G, P, L, "span 70", True)
        fb1 = e.tick_light_fallbacks()
        # more groups listed than the fallback grid (max(2,048, 2 x the previous count)) has workgroups
        assert fb1 > max(2048, 2 * fb0), (fb0, fb1, _active(gf))
        for k in range(3):
            _step(e, o, lp, G, P, L, f"steady again {k}", False)
            _start_all(e, o, lp, G, P, rng, 1)


@pytest.mark.parametrize("P", [4, 5, 6, 7, 8])
def test_light_few_successes_gpu(P):
    """Groups where fewer than P/2 followers reply success and the others sit
    ahead of the leader's nextIndex (prev below their dummy: IC_BELOW, the
    reply dropped by the leader's gate, raft_append_entry.go:123-127): a1 runs
    on an order statistic that still holds the others' older matchIndex
    (:78, :89-105). The light launch settles the group when that statistic
    cannot pass commitIndex or its top's term settles a1 (currentTerm, or
    below it under terms_sorted), and lists it otherwise; the leader's
    matchIndex words for those followers are drawn around commitIndex so
    each happens, and some successes lower their word (old matchIndex above
    last), where only the bound applies."""
    G, L = 1024, 256
    rng = np.random.default_rng(7700 + P)
    st, lp, _ = synth_tick_state(G, P, L, seed=7700 + P)
    o = Oracle(G, P, L, st)
    for _ in range(3):  # steady on the oracle: followers caught up
        o.replicate_tick(lp)
        g = np.flatnonzero(lp >= 0)
        o.start((g * P + lp[g]).astype(np.int32), rng.integers(1, 4, size=len(g)).astype(np.int32))
    o.replicate_tick(lp)
    s = {k: v.copy() for k, v in o.state().items()}
    nx = s["next_index"].reshape(G * P, P)
    mt = s["match_index"].reshape(G * P, P)
    dm, hd, la, cm = s["dummy_index"], s["log_head"], s["last_index"], s["commit_index"]
    changed = 0
    for g in np.flatnonzero(lp >= 0)[::2]:
        ld = g * P + lp[g]
        fol = [j for j in range(P) if j != lp[g]]
        nsucc = int(rng.integers(1, P // 2))  # 1 .. P/2 - 1 successes
        ahead = rng.permutation(fol)[: len(fol) - nsucc]
        ok = True
        for j in ahead:
            f = g * P + j
            # the follower compacted to its last entry (ring mapping kept), the
            # leader's nextIndex one below that dummy
            if la[f] - 1 < dm[ld] or la[f] <= dm[f]:
                ok = False
                break
        if not ok:
            continue
        for j in ahead:
            f = g * P + j
            hd[f] = (hd[f] + (la[f] - dm[f])) % L
            dm[f] = la[f]
            cm[f] = max(cm[f], dm[f])
            nx[ld, j] = dm[f]
            mt[ld, j] = max(0, cm[ld] + int(rng.integers(-3, 4)))
        if rng.random() < 0.3:  # a success that lowers its matchIndex word (a bad-state leader)
            sj = [j for j in fol if j not in set(ahead)][0]
            mt[ld, sj] = la[ld] + 2
        changed += 1
    assert changed > 50
    o2 = Oracle(G, P, L, s)
    with Engine(G, P, L) as e:
        e.load_state(s)
        e.set_tick_mode(TICK_LIGHT)
        for k in range(3):
            gf = _step(e, o2, lp, G, P, L, f"few P={P} step {k}", export=(k == 1))
            if k == 0:
                fb = e.tick_light_fallbacks()
                assert 0 <= fb < changed, (fb, changed)  # some of them settled in the light launch
            _start_all(e, o2, lp, G, P, rng, 3)


@pytest.mark.parametrize("j", [0, 5])
def test_light_top_of_index_domain_gpu(j):
    """Steady ticks whose Indexes end within j of 2^31 - 2 (include/mraft.h: the
    Index domain): the light launch's entry loop and ring arithmetic there."""
    G, P, L, steps, cmax = 512, 5, 256, 6, 3
    st0, lp, _ = synth_tick_state(G, P, L, seed=5150 + j)
    st = shift_indices(st0, top_offset(st0, j + steps * cmax))
    fbs = _steady_run(G, P, L, 5150 + j, 2, steps, cmax=cmax, state=st, lp=lp)
    assert fbs[-1][0] < fbs[-1][1], fbs


def test_light_mode_calls_and_p1_gpu():
    """The mode calls (MRAFT_TICK_AUTO by default, bad modes rejected, the mode
    kept across shard changes) and P = 1, where the one-lane-per-group tick
    already is the light form."""
    G, P, L = 64, 1, 16
    st, lp, _ = synth_tick_state(G, P, L, seed=3)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        assert e.tick_mode() == TICK_AUTO  # the default
        with pytest.raises(MraftError):
            e.set_tick_mode(3)
        e.set_tick_mode(TICK_LIGHT)
        e.set_tick_shards(2)
        assert e.tick_mode() == TICK_LIGHT
        for k in range(2):
            _step(e, o, lp, G, P, L, f"P=1 step {k}", bool(k))
        e.set_tick_mode(TICK_FULL)
        _step(e, o, lp, G, P, L, "P=1 full", False)


@pytest.mark.parametrize("shards", [1, 2])
def test_auto_mode_gpu(shards):
    """MRAFT_TICK_AUTO: a heavy first tick (every group of the seeded state
    falls back) turns the engine to the full tick, a light tick every 32nd
    re-measures, and the steady state brings the light tick back — the oracle
    equal after every one of 40 ticks with Start() between them."""
    G, P, L = 512, 5, 256
    rng = np.random.default_rng(31 + shards)
    st, lp, _ = synth_tick_state(G, P, L, seed=2024 + shards)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.set_tick_shards(shards)
        e.set_tick_mode(TICK_AUTO)
        assert e.tick_mode() == TICK_AUTO
        seen = set()
        for k in range(40):
            _step(e, o, lp, G, P, L, f"auto step {k}", bool(k % 3 == 0))
            seen.add(e.tick_light_fallbacks())
            _start_all(e, o, lp, G, P, rng, 2)
        assert len(seen) > 1 and min(seen) >= 0, seen  # light ticks ran and were counted again


def _oracle_start_and_tick(o, lp, counts, G, P):
    """mraft_start over the groups' leader slots (counts != 0, leader_peer in
    range), then the tick: the composition mraft_start_and_tick must equal."""
    idx, term = np.full(G, -1, np.int32), np.full(G, -1, np.int32)
    isl, err = np.zeros(G, np.int32), np.zeros(G, np.int32)
    sel = np.flatnonzero((lp >= 0) & (lp < P) & (counts != 0))
    if len(sel):
        oi, ot, ol, oe = o.start((sel * P + lp[sel]).astype(np.int32), counts[sel].astype(np.int32))
        idx[sel], term[sel], isl[sel], err[sel] = oi, ot, ol, oe
    err[(lp >= P) & (counts != 0)] = 6  # MRAFT_ITEM_BAD_SLOT
    return o.replicate_tick(lp), (idx, term, isl, err)


@pytest.mark.parametrize("mode,P,shards", [(TICK_LIGHT, 5, 1), (TICK_LIGHT, 8, 2), (TICK_FULL, 5, 1),
                                           (TICK_AUTO, 3, 2), (TICK_LIGHT, 2, 3), (TICK_AUTO, 1, 1)])
def test_start_and_tick_gpu(mode, P, shards):
    """mraft_start_and_tick (raft.go:90-104 at every group's leader, then the
    tick) == mraft_start over those slots followed by mraft_replicate_tick on
    the oracle, over ten steps: counts 0-4 with some negative (MRAFT_ITEM_BAD_SLOT)
    and some past the ring's capacity (MRAFT_ITEM_LOG_FULL), leader moves,
    idle and out-of-range leader_peer; Start inside the light launch (the
    followers' copies of the new entries and a1's probe from currentTerm),
    and as its own launch on the full tick's path."""
    G, L = 700, 128
    rng = np.random.default_rng(4400 + 10 * P + shards + mode)
    st, lp, _ = synth_tick_state(G, P, L, seed=4400 + P)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.set_tick_shards(min(shards, G))
        e.set_tick_mode(mode)
        for k in range(10):
            counts = rng.integers(0, 5, size=G).astype(np.int32)
            counts[rng.random(G) < 0.03] = -1
            counts[rng.random(G) < 0.02] = L  # past any ring's capacity
            lpk = lp.copy()
            lpk[rng.random(G) < 0.03] = -1
            lpk[rng.random(G) < 0.01] = P
            gf, outs = e.start_and_tick(lpk, counts)
            ogf, oouts = _oracle_start_and_tick(o, lpk, counts, G, P)
            for a, b, name in zip(outs, oouts, ("index", "term", "is_leader", "err")):
                assert np.array_equal(a, b), (k, name)
            assert np.array_equal(gf, ogf), (k, "group flags")
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"start_and_tick step {k}")
            moved = rng.random(G) < 0.05
            lp = np.where(moved, rng.integers(0, P, size=G), lp).astype(np.int32)
