"""Persistence (SURVEY.md §5 checkpoint/resume, §8f #4): the persist_dirty
set of every entry point against the oracle's persist() call sites, SaveState
read-out, Make + readPersist restore, and the Persister flush / restart
driver. CPU tests run on the oracle; `gpu` tests run libmraft_hip.so against
it through the C ABI."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal

from multiraft_amd import synth_election_state, synth_seed, synth_tick_state
from multiraft_amd._abi import ITEM_BAD_SLOT, ITEM_DUP_SLOT, ITEM_LOG_FULL, PERSISTENT
from multiraft_amd.engine import decode_persistent, encode_persistent
from multiraft_amd.persister import Persister, flush_persist, restart


def _engine(G, P, L, st):
    from multiraft_amd import Engine
    e = Engine(G, P, L)
    e.load_state(st)
    return e


def _restore_batch(G, P, L, rng):
    """Persistent records for a few slots, with bad / oversize / dup items."""
    slots = rng.choice(G * P, size=min(12, G * P), replace=False).astype(np.int32)
    hdr = np.zeros(len(slots) + 3, dtype=PERSISTENT)
    parts, off = [], 0
    for i, s in enumerate(slots):
        d = int(rng.integers(0, 50))
        n = int(rng.integers(1, L + 1))
        hdr[i] = (s, int(rng.integers(0, 99)), int(rng.integers(-1, P)), d, d + n - 1, 0, off)
        parts.append(np.sort(rng.integers(0, 9, n)).astype(np.int32))
        off += n
    hdr[-3] = (G * P, 1, -1, 0, 0, 0, 0)              # bad slot
    hdr[-2] = (slots[0], 1, -1, 0, L, 0, 0)           # L + 1 entries
    hdr[-1] = (slots[1], 1, -1, 0, 0, 0, 0)           # duplicate slot
    return hdr, np.concatenate(parts)


def test_tick_marks_every_handled_follower_and_step_down_oracle():
    G, P, L = 64, 5, 64
    st, lp, ic = synth_tick_state(G, P, L, seed=31)
    o = Oracle(G, P, L, st)
    o.replicate_tick(lp)
    bits = o.collect_persist()
    assert not o.collect_persist().any()               # cleared on read
    # every follower item that reached HandleAppendEntries persisted (deferred :111)
    followers = np.array([s for s in range(G * P) if s % P != lp[s // P]])
    assert bits[followers].all()
    assert set(np.unique(bits)) <= {0, 1, 3}


def test_restore_and_read_oracle():
    G, P, L = 8, 3, 16
    rng = np.random.default_rng(5)
    st, _, _ = synth_tick_state(G, P, L, seed=32)
    o = Oracle(G, P, L, st)
    hdr, terms = _restore_batch(G, P, L, rng)
    err = o.restore(hdr, terms)
    assert err[-3] == ITEM_BAD_SLOT and err[-2] == ITEM_LOG_FULL and err[-1] == ITEM_DUP_SLOT
    assert not err[:-3].any()
    h2, t2 = o.read_persistent(hdr["slot"][:-3])
    for f in ("slot", "current_term", "voted_for", "dummy_index", "last_index"):
        assert np.array_equal(h2[f], hdr[f][:-3]), f
    assert np.array_equal(t2, terms)
    s = o.state()
    sl = hdr["slot"][:-3]
    assert (s["state"][sl] == 3).all() and np.array_equal(s["commit_index"][sl], hdr["dummy_index"][:-3])


def test_flush_restart_round_trip_oracle():
    G, P, L = 16, 5, 32
    st, lp, _ = synth_tick_state(G, P, L, seed=33)
    o = Oracle(G, P, L, st)
    o.replicate_tick(lp)
    per = Persister(G * P)
    flushed = flush_persist(o, per)
    assert len(flushed) > 0
    before = o.store_state()
    err = restart(o, per, flushed)
    assert not err.any()
    after = o.state()
    for f in ("current_term", "voted_for", "dummy_index", "last_index"):
        assert np.array_equal(after[f][flushed], before[f][flushed]), f
    for s in flushed:
        n = before["last_index"][s] - before["dummy_index"][s] + 1
        assert np.array_equal(after["log_term"][s * L:s * L + n], before["log_term"][s * L:s * L + n])
        rec, t = decode_persistent(per.read_raft_state(int(s)))
        assert int(rec["current_term"]) == before["current_term"][s] and len(t) == n


@pytest.mark.gpu
@pytest.mark.parametrize("G,P,L,seed", [(96, 3, 64, 41), (64, 5, 256, 42), (32, 7, 96, 43)])
def test_tick_persist_gpu(G, P, L, seed):
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        for k in range(2):
            assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp))
            assert_states_equal(e.store_state(), o.state(), G, P, L, f"tick {k}")
            assert np.array_equal(e.collect_persist(), o.collect_persist())
            assert not e.collect_persist().any()


@pytest.mark.gpu
def test_election_storm_persist_gpu():
    G, P, L, R = 512, 7, 64, 8
    st, mask = synth_election_state(G, P, L, seed=synth_seed(5), rounds=R)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert np.array_equal(e.election_rounds(mask), o.election_rounds(mask))
        assert np.array_equal(e.collect_persist(), o.collect_persist())
        assert_states_equal(e.store_state(), o.state(), G, P, L, "storm")


@pytest.mark.gpu
def test_read_restore_gpu():
    G, P, L = 64, 5, 128
    rng = np.random.default_rng(44)
    st, lp, _ = synth_tick_state(G, P, L, seed=45)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        slots = rng.choice(G * P, 40, replace=False).astype(np.int32)
        he, te = e.read_persistent(slots)
        ho, to = o.read_persistent(slots)
        assert np.array_equal(he, ho) and np.array_equal(te, to)
        hdr, terms = _restore_batch(G, P, L, rng)
        assert np.array_equal(e.restore(hdr, terms), o.restore(hdr, terms))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "restore")
        # the restored replicas keep working: a tick on the restored state
        assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "tick after restore")


@pytest.mark.gpu
def test_flush_restart_gpu():
    G, P, L = 256, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=46)
    o = Oracle(G, P, L, st)
    pe, po_ = Persister(G * P), Persister(G * P)
    with _engine(G, P, L, st) as e:
        e.replicate_tick(lp)
        o.replicate_tick(lp)
        fe, fo = flush_persist(e, pe), flush_persist(o, po_)
        assert np.array_equal(fe, fo)
        assert all(pe.read_raft_state(int(s)) == po_.read_raft_state(int(s)) for s in fe)
        crash = fe[::3]
        assert np.array_equal(restart(e, pe, crash), restart(o, po_, crash))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "restart")


def test_encode_matches_read_persistent_oracle():
    G, P, L = 4, 3, 16
    st, _, _ = synth_tick_state(G, P, L, seed=47)
    o = Oracle(G, P, L, st)
    hdr, terms = o.read_persistent(np.arange(G * P, dtype=np.int32))
    for i in range(G * P):
        n = int(hdr["last_index"][i] - hdr["dummy_index"][i] + 1)
        off = int(hdr["terms_offset"][i])
        b = encode_persistent(hdr[i], terms[off:off + n])
        rec, t = decode_persistent(b)
        assert np.array_equal(t, terms[off:off + n])
        assert int(rec["last_index"]) == int(hdr["last_index"][i])
