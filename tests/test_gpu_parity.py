"""GPU parity: libmraft_hip.so on an MI355X against the CPU oracle, bit for
bit, through the C ABI (multiraft_amd.engine over ctypes)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

from kat_runner import kat_state, load_kats, run_kat  # noqa: E402
from make_golden import check_kat  # noqa: E402
from oracle_lib import Oracle, assert_states_equal  # noqa: E402

from multiraft_amd import (Engine, entry_positions, synth_fold_batch, synth_seed, synth_tick_state,  # noqa: E402
                           )
from multiraft_amd.engine import export_group_status_into  # noqa: E402
from multiraft_amd._abi import AE_ARGS, AE_RESULT, RV_ARGS, RV_RESULT  # noqa: E402

pytestmark = pytest.mark.gpu
KATS = load_kats()


def _engine(G, P, L, st):
    e = Engine(G, P, L)
    e.load_state(st)
    return e


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_kat_gpu(k):
    with _engine(k["G"], k["P"], k["L"], kat_state(k)) as e:
        check_kat(k, run_kat(k, e, e.store_state))


@pytest.mark.parametrize("G,P,L,seed", [(48, 3, 64, 1), (32, 5, 128, 2), (24, 7, 96, 3),
                                        (40, 2, 32, 4), (30, 4, 16, 5), (16, 8, 64, 6),
                                        (20, 1, 16, 7), (64, 5, 8, 8), (1000, 6, 40, 9)])
def test_tick_small(G, P, L, seed):
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    lp = lp.copy()
    lp[::7] = -1
    if G > 9 and P > 1:
        lp[9] = P
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        cnt_gpu = e.replicate_tick_count(lp)
        assert cnt_gpu == o.replicate_tick_count(lp)
        gf = e.replicate_tick(lp)
        ogf = o.replicate_tick(lp)
        assert np.array_equal(gf, ogf)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "tick")


@pytest.mark.parametrize("cfg", ["c2", "c3_small", "c3_fullL"])
def test_tick_configs(cfg):
    G, P, L = {"c2": (1024, 3, 256), "c3_small": (2048, 5, 1024), "c3_fullL": (4096, 5, 4096)}[cfg]
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(2 if cfg == "c2" else 3))
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        gf = e.replicate_tick(lp)
        assert np.array_equal(gf, o.replicate_tick(lp, nthreads=8))
        assert_states_equal(e.store_state(), o.state(), G, P, L, cfg)
        # a second tick on the evolved state (catch-up continuation)
        gf2 = e.replicate_tick(lp)
        assert np.array_equal(gf2, o.replicate_tick(lp, nthreads=8))
        assert_states_equal(e.store_state(), o.state(), G, P, L, cfg + " tick 2")


def test_fold_batch_config2():
    G, P, L = 1024, 3, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(2))
    items, seg = synth_fold_batch(st, G, P, L, lp, seed=synth_seed(2))
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        f, err = e.process_append_replies(items, seg)
        of, oerr = o.process_append_replies(items, seg)
        assert np.array_equal(err, oerr) and np.array_equal(f, of)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "fold")


def test_fold_far_bad_slot_gpu():
    """A segment whose slot lies far outside the image is rejected without
    reading any replica state (the fold never dereferences it); the other
    segments of the batch fold as on the oracle."""
    G, P, L = 1024, 3, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(2))
    items, seg = synth_fold_batch(st, G, P, L, lp, seed=synth_seed(2))
    items = items.copy()
    bad = slice(int(seg[7]), int(seg[8]))
    items["slot"][bad] = 1 << 30
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        f, err = e.process_append_replies(items, seg)
        of, oerr = o.process_append_replies(items, seg)
        assert (err[bad] == 6).all() and (f[bad] == 0).all()  # MRAFT_ITEM_BAD_SLOT
        assert np.array_equal(err, oerr) and np.array_equal(f, of)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "fold bad slot")


def test_fold_dup_empty_uncovered_gpu():
    """Segments that repeat a leader slot (the lowest wins, the others are
    MRAFT_ITEM_DUP_SLOT with no state change), empty segments, and items no
    segment covers (flag 0, error 0): the claim and the outputs' zeroing run
    in one launch, the duplicate check inside the fold."""
    G, P, L = 1024, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    items, seg = synth_fold_batch(st, G, P, L, lp, seed=synth_seed(3))
    nseg = len(seg) - 1
    parts, bounds = [items[:3]], [3]                     # 3 uncovered items first
    for k in range(nseg):
        parts.append(items[int(seg[k]):int(seg[k + 1])])
        bounds.append(bounds[-1] + len(parts[-1]))
        if k % 7 == 3:                                   # the same leader again, later in the batch
            parts.append(items[int(seg[k]):int(seg[k + 1])][::-1])
            bounds.append(bounds[-1] + len(parts[-1]))
        if k % 11 == 5:                                  # an empty segment
            bounds.append(bounds[-1])
    parts.append(items[:4])                              # 4 uncovered items last
    it2 = np.concatenate(parts)
    sb = np.array(bounds, np.int64)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        f, err = e.process_append_replies(it2, sb)
        of, oerr = o.process_append_replies(it2, sb)
        assert (err == 5).any() and (err == 0).any()     # MRAFT_ITEM_DUP_SLOT
        assert (err[:3] == 0).all() and (f[:3] == 0).all() and (err[-4:] == 0).all() and (f[-4:] == 0).all()
        assert np.array_equal(err, oerr) and np.array_equal(f, of)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "fold dup")


@pytest.mark.parametrize("P,seed", [(5, 24), (3, 25), (8, 26), (2, 27)])
def test_fold_long_segments_gpu(P, seed):
    """Segments longer than one 64-reply batch, repeated peers, many a1
    evaluations per segment (ranges probed in parallel, Figure-8 scans)."""
    from oracle_lib import random_reply_segments
    G, L = 64, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    items, seg = random_reply_segments(st, G, P, lp, seed=seed)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        f, err = e.process_append_replies(items, seg)
        of, oerr = o.process_append_replies(items, seg)
        assert np.array_equal(err, oerr) and np.array_equal(f, of)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "fold long")


@pytest.mark.parametrize("P,seed", [(5, 34), (3, 35), (8, 36)])
def test_fold_short_segments_gpu(P, seed):
    """Segments of at most eight replies (the eight-segments-per-wave fold),
    several a1 evaluations each, so one segment's pending ranges land in
    different k_fold_tail scan waves and the replica's commitIndex is the maximum
    of their hits and the probes' (atomicMax); Figure-8 logs included."""
    from oracle_lib import random_reply_segments
    G, L = 1024, 512
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    items, seg = random_reply_segments(st, G, P, lp, seed=seed, max_len=8)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        f, err = e.process_append_replies(items, seg)
        of, oerr = o.process_append_replies(items, seg)
        assert np.array_equal(err, oerr) and np.array_equal(f, of)
        assert (f & 2).any()  # MRAFT_F_COMMITTED: some evaluations commit
        assert_states_equal(e.store_state(), o.state(), G, P, L, "fold short")


def test_item_path_gpu():
    G, P, L = 256, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=61)
    o = Oracle(G, P, L, st)
    slots = np.array([g * P + lp[g] for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    peers = np.array([p for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    with _engine(G, P, L, st) as e:
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(gerr, ogerr) and np.array_equal(args, oargs)
        ok = gerr == 0
        # entries from an external buffer (the network case): copy them out
        ent = []
        a2 = args[ok].copy()
        off = 0
        for j, a in enumerate(args[ok]):
            # entries_offset is a logical ring position: unrolled through log_head
            ent.append(st["log_term"][entry_positions(st["log_head"], L, [a["entries_offset"]], [a["n_entries"]])])
            a2["entries_offset"][j] = off
            off += a["n_entries"]
        ent = np.concatenate(ent + [np.zeros(1, np.int32)]).astype(np.int32)
        rep, herr = e.handle_append_entries(a2, ent)
        orep, oherr = o.handle_append_entries(a2, ent)
        assert np.array_equal(herr, oherr) and np.array_equal(rep, orep)
        res = np.zeros(int(ok.sum()), dtype=AE_RESULT)
        res["slot"], res["peer"] = slots[ok], peers[ok]
        res["args_term"], res["args_prev_log_index"] = args["term"][ok], args["prev_log_index"][ok]
        res["args_n_entries"] = args["n_entries"][ok]
        res["reply_term"], res["reply_success"] = rep["term"], rep["success"]
        res["reply_conflict_index"] = rep["conflict_index"]
        res = res[herr == 0]
        seg = np.concatenate([[0], np.cumsum(np.bincount(res["slot"] // P, minlength=G))]).astype(np.int64)
        f, ferr = e.process_append_replies(res, seg)
        of, oferr = o.process_append_replies(res, seg)
        assert np.array_equal(f, of) and np.array_equal(ferr, oferr)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "item path")


def test_dup_and_bad_slots_gpu():
    G, P, L = 4, 3, 16
    st, lp, _ = synth_tick_state(G, P, L, seed=51)
    a = np.zeros(4, dtype=AE_ARGS)
    a["slot"] = [1, 1, 99, 1]
    a["term"] = 1
    with _engine(G, P, L, st) as e:
        rep, err = e.handle_append_entries(a, np.zeros(4, np.int32))
        assert err.tolist() == [0, 5, 6, 5]


def test_elections_gpu():
    from test_oracle import _random_vote_state
    G, P, L = 512, 7, 16
    rng = np.random.default_rng(7)
    st = _random_vote_state(G, P, L, 71)
    o = Oracle(G, P, L, st)
    cands = np.array([g * P + rng.integers(0, P) for g in range(G)], np.int32)
    with _engine(G, P, L, st) as e:
        args, err = e.start_election(cands)
        oargs, oerr = o.start_election(cands)
        assert np.array_equal(args, oargs) and np.array_equal(err, oerr)
        rv = np.zeros(G * (P - 1), dtype=RV_ARGS)
        res = np.zeros(G * (P - 1), dtype=RV_RESULT)
        i = 0
        for g, c in enumerate(cands):
            for p in range(P):
                v = g * P + p
                if v == c:
                    continue
                a = args[g]
                lt = a["last_log_term"] if rng.random() > 0.2 else rng.integers(0, 6)
                rv[i] = (v, a["candidate_id"], a["term"], a["last_log_index"], lt)
                res[i] = (c, p, a["term"], 0, 0)
                i += 1
        rep, rerr = e.handle_request_vote(rv)
        orep, orerr = o.handle_request_vote(rv)
        assert np.array_equal(rep, orep) and np.array_equal(rerr, orerr)
        res["reply_term"], res["vote_granted"] = rep["term"], rep["vote_granted"]
        seg = np.arange(0, len(res) + 1, P - 1, dtype=np.int64)
        f, ferr = e.process_vote_replies(res, seg)
        of, oferr = o.process_vote_replies(res, seg)
        assert np.array_equal(f, of) and np.array_equal(ferr, oferr)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "elections")
        c, tl = e.export_group_status(cands % P)
        oc, otl = o.export_group_status(cands % P)
        assert np.array_equal(c, oc) and np.array_equal(tl, otl)


@pytest.mark.parametrize("P,L,mono", [(2, 8, False), (3, 16, False), (5, 12, False), (5, 16, True),
                                      (7, 10, False), (8, 9, False), (4, 64, False), (5, 256, False),
                                      (5, 1024, True)])
def test_tick_random_adversarial_gpu(P, L, mono):
    """Arbitrary (not reachable-shaped) states: non-monotone terms, accidental
    matches, snapshots, panics, near-capacity logs, bad states."""
    from random_states import random_tick_state
    rng = np.random.default_rng(2000 + P * 100 + L)
    G = 700
    st, lp = random_tick_state(rng, G, P, L, monotone=mono)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        gf = e.replicate_tick(lp)
        assert np.array_equal(gf, o.replicate_tick(lp))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "adversarial tick")


@pytest.mark.parametrize("P,L", [(2, 8), (3, 16), (5, 12), (5, 256), (8, 40), (5, 1024)])
def test_tick_snapshot_heavy_gpu(P, L):
    """InstallSnapshot inside the fused tick: stale, outdated, new-log and
    sliced installs, dropped-on-panic items, and the fold's match/next update."""
    from random_states import random_tick_state
    rng = np.random.default_rng(2500 + P * 100 + L)
    G = 700
    st, lp = random_tick_state(rng, G, P, L, snap=True)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        gf = e.replicate_tick(lp)
        ogf = o.replicate_tick(lp)
        assert np.array_equal(gf, ogf)
        assert (ogf & 256).any()
        assert_states_equal(e.store_state(), o.state(), G, P, L, "snapshot-heavy tick")


@pytest.mark.parametrize("P,R", [(3, 16), (5, 8), (7, 64), (8, 5), (2, 7), (1, 3)])
def test_election_rounds_gpu(P, R):
    from multiraft_amd import synth_election_state
    G, L = 2048, 8
    st, mask = synth_election_state(G, P, L, seed=300 + P, rounds=R)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        gf = e.election_rounds(mask)
        assert np.array_equal(gf, o.election_rounds(mask))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "election rounds")


@pytest.mark.parametrize("P,L", [(3, 16), (5, 12), (7, 32), (5, 300)])
def test_snapshot_install_gpu(P, L):
    from random_states import random_tick_state
    from snapshot_cases import run_snapshot_scenario
    G = 400
    rng = np.random.default_rng(700 + P + L)
    st, lp = random_tick_state(rng, G, P, L)
    lp = np.where((lp >= 0) & (lp < P), lp, 0).astype(np.int32)
    o = Oracle(G, P, L, st)
    oo = run_snapshot_scenario(o, st, G, P, L, lp, seed=9)
    with _engine(G, P, L, st) as e:
        go = run_snapshot_scenario(e, st, G, P, L, lp, seed=9)
        for k in oo:
            assert np.array_equal(go[k], oo[k]), k
        assert_states_equal(e.store_state(), o.state(), G, P, L, "snapshot scenario")


@pytest.mark.parametrize("G,P,L,seed", [(96, 5, 64, 61), (40, 3, 32, 62), (16, 1, 16, 63)])
def test_tick_export_fused_gpu(G, P, L, seed):
    """mraft_replicate_tick_export == the tick followed by GetState export,
    idle (-1) and out-of-range leader indices included."""
    st, lp, _ = synth_tick_state(G, P, L, seed=seed)
    lp = lp.copy()
    lp[::5] = -1
    lp[3] = P
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        gf, c, tl = e.replicate_tick_export(lp)
        assert np.array_equal(gf, o.replicate_tick(lp))
        oc, otl = o.export_group_status(lp)
        assert np.array_equal(c, oc) and np.array_equal(tl, otl)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "tick+export")


def _assert_big_states_equal(a, b, G, P, L, ctx, rows=8192):
    """assert_states_equal in row blocks (the full config-#3 image is 5 GiB)."""
    for k in a:
        if k != "log_term":
            assert np.array_equal(a[k], b[k]), f"{ctx}: {k}"
    la, lb = a["log_term"].reshape(G * P, L), b["log_term"].reshape(G * P, L)
    live = a["last_index"] - a["dummy_index"]
    col = np.arange(L)[None, :]
    for r0 in range(0, G * P, rows):
        m = col <= live[r0:r0 + rows, None]
        assert np.array_equal(np.where(m, la[r0:r0 + rows], 0), np.where(m, lb[r0:r0 + rows], 0)), \
            f"{ctx}: log rows {r0}..{r0 + rows}"


def test_tick_full_config3_gpu():
    """BASELINE config #3 at full size (65,536 groups x 5 peers x 4,096-entry
    logs, the bench workload): two ticks bit-exact against the oracle (state,
    persist bits, group flags, fused GetState words) and the algorithmic word
    count of the roofline equal to the oracle's instrumented count."""
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        for k in range(2):
            gf, c, tl = e.replicate_tick_export(lp)
            assert np.array_equal(gf, o.replicate_tick(lp, nthreads=16)), f"tick {k} flags"
            oc, otl = o.export_group_status(lp)
            assert np.array_equal(c, oc) and np.array_equal(tl, otl)
            _assert_big_states_equal(e.store_state(), o.state(), G, P, L, f"full tick {k}")


def test_tick_full_config4_one_gpu():
    """BASELINE config #4 as its N=1 point (`bench.py --global-groups 262144`):
    all 262,144 groups x 5 peers x 4,096-entry logs (21.5 GB of logs) on one
    GPU, one tick bit-exact against the oracle (state, persist bits, group
    flags, fused GetState words), and the roofline's word count."""
    G, P, L = 262144, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=16)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        del st
        assert e.replicate_tick_count(lp) == o.replicate_tick_count(lp)
        gf, c, tl = e.replicate_tick_export(lp)
        assert np.array_equal(gf, o.replicate_tick(lp, nthreads=16)), "config #4 tick flags"
        oc, otl = o.export_group_status(lp)
        assert np.array_equal(c, oc) and np.array_equal(tl, otl)
        _assert_big_states_equal(e.store_state(), o.state(), G, P, L, "config #4 tick")


def test_election_storm_full_config5_gpu():
    """BASELINE config #5 at full size: 65,536 groups x 7 peers, 64 rounds."""
    from multiraft_amd import synth_election_state
    G, P, L, R = 65536, 7, 8, 64
    st, mask = synth_election_state(G, P, L, seed=synth_seed(5), rounds=R)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert np.array_equal(e.election_rounds(mask), o.election_rounds(mask))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "full storm")


def test_start_and_applier_gpu():
    """Start (raft.go:90-104) on random slots — leaders and non-leaders,
    duplicate slots, multi-entry counts, appends past the capacity — then the
    applier's ranges (raft.go:153-203) after a tick, against the oracle."""
    G, P, L = 128, 5, 64
    rng = np.random.default_rng(71)
    st, lp, _ = synth_tick_state(G, P, L, seed=72)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        for _ in range(3):
            slots = rng.integers(0, G * P, 200).astype(np.int32)
            counts = rng.integers(1, 24, 200).astype(np.int32)
            counts[::17] = 0                                   # rejected: BAD_SLOT
            got = e.start(slots, counts)
            exp = o.start(slots, counts)
            for a, b in zip(got, exp):
                assert np.array_equal(a, b)
            assert_states_equal(e.store_state(), o.state(), G, P, L, "start")
        assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp))
        for _ in range(2):
            fr, to = e.collect_apply()
            ofr, oto = o.collect_apply()
            assert np.array_equal(fr, ofr) and np.array_equal(to, oto)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "applier")


@pytest.mark.parametrize("cap", [None, 37])
def test_applier_compact_gpu(cap):
    """The compacted applier lists exactly the slots whose range is non-empty,
    ascending, with the dense applier's ranges; with a short buffer only the
    listed slots advance, and a second call returns the rest."""
    G, P, L = 700, 5, 64
    st, lp, _ = synth_tick_state(G, P, L, seed=81)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp))
        pre = e.store_state()
        fr, to = o.collect_apply()
        want = np.nonzero(to >= fr)[0]
        sl, f, t, n = e.collect_apply_compact(cap)
        assert n == len(want) and n > 40
        k = len(sl)
        assert k == (n if cap is None else min(cap, n))
        assert np.array_equal(sl, want[:k]) and np.array_equal(f, fr[want[:k]]) and np.array_equal(t, to[want[:k]])
        got = e.store_state()
        exp_applied = pre["last_applied"].copy()
        exp_applied[want[:k]] = pre["commit_index"][want[:k]]
        assert np.array_equal(got["last_applied"], exp_applied)
        if cap is not None:
            sl2, f2, t2, n2 = e.collect_apply_compact()
            assert n2 == n - k and np.array_equal(sl2, want[k:])
        assert e.collect_apply_compact()[3] == 0
        assert_states_equal(e.store_state(), o.state(), G, P, L, "applier compact")


def test_applier_compact_snapshot_outputs_gpu():
    """The compacted applier without snapshot outputs behaves as the dense
    one without them: only commitIndex > lastApplied slots are listed and a
    pending SnapshotValid (hasSnapshot, raft.go:168-177) stays for the call
    that takes it; that call lists it first, with the dummy's Index and Term."""
    G, P, L = 300, 5, 64
    st, lp, _ = synth_tick_state(G, P, L, seed=82)
    rng = np.random.default_rng(3)
    hs = rng.random(G * P) < 0.2
    st["has_snapshot"] = hs.astype(np.int32)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        ofr, oto = o.collect_apply()                        # dense, no snapshot outputs
        want = np.nonzero(oto >= ofr)[0]
        sl, f, t, n = e.collect_apply_compact()
        assert n == len(want) and np.array_equal(sl, want)
        assert np.array_equal(f, ofr[want]) and np.array_equal(t, oto[want])
        assert np.array_equal(e.store_state()["has_snapshot"], st["has_snapshot"])   # untouched
        ofr, oto, osi, ost = o.collect_apply(snapshots=True)
        want = np.nonzero((oto >= ofr) | (osi >= 0))[0]
        sl, si, stm, f, t, n = e.collect_apply_compact(snapshots=True)
        assert n == len(want) == int(hs.sum()) and np.array_equal(sl, want)
        assert np.array_equal(si, osi[want]) and np.array_equal(stm, ost[want])
        assert not e.store_state()["has_snapshot"].any()
        assert_states_equal(e.store_state(), o.state(), G, P, L, "applier compact, snapshots")


@pytest.mark.parametrize("S,G", [(2, 4096), (3, 4099), (8, 1031)])
def test_tick_shards_on_engine_queues_gpu(S, G):
    """mraft_set_tick_shards: one engine splits every tick into S contiguous
    group ranges on S hardware queues it owns (uneven ranges when S does not
    divide G); several ticks over fresh copies overlap on the queues, a
    following one-launch call (the export) joins them, and every copy's flags,
    export words and state equal the oracle's (compared directly, not only
    against one launch)."""
    import torch

    from multiraft_amd import DEVICE

    P, L, C = 5, 256, 3
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    lp_d = torch.from_numpy(lp).to(dev)
    copies = [{k: v.clone() for k, v in master.items()} for _ in range(C)]
    flags = [torch.zeros(G, dtype=torch.int32, device=dev) for _ in range(C)]
    exp = [torch.zeros(2 * G, dtype=torch.int32, device=dev) for _ in range(C)]
    after = [torch.zeros(2 * G, dtype=torch.int32, device=dev) for _ in range(C)]
    torch.cuda.synchronize()
    with Engine(G, P, L, alloc=False) as e:
        e.set_tick_shards(S)
        assert e.tick_shards() == S and all(e.shard_stream(s) for s in range(S)) and not e.shard_stream(S)
        for c in range(C):
            e.bind(copies[c])
            e.replicate_tick_export(lp_d, flags[c], exp[c][:G], exp[c][G:], where=DEVICE)
        for c in range(C):  # joins the shards: reads every copy's post-tick state
            e.bind(copies[c])
            export_group_status_into(e, lp_d, after[c][:G], after[c][G:])
        e.synchronize()
    o = Oracle(G, P, L, st)
    of = o.replicate_tick(lp)
    oc, ot = o.export_group_status(lp)
    for c in range(C):
        assert np.array_equal(flags[c].cpu().numpy(), of), c
        assert np.array_equal(exp[c][:G].cpu().numpy(), oc) and np.array_equal(exp[c][G:].cpu().numpy(), ot)
        assert np.array_equal(after[c][:G].cpu().numpy(), oc) and np.array_equal(after[c][G:].cpu().numpy(), ot)
        got = {k: v.cpu().numpy() for k, v in copies[c].items()}
        assert_states_equal(got, o.state(), G, P, L, f"sharded tick, copy {c}")


def test_tick_shards_host_buffers_and_reset_gpu():
    """A host-buffer tick with shards (staged on the engine stream, forked,
    joined before the copy-back), then shards = 1 again: both equal the
    oracle's ticks."""
    G, P, L = 2048, 5, 128
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3) + 7)
    o = Oracle(G, P, L, st)
    with _engine(G, P, L, st) as e:
        e.set_tick_shards(4)
        f1, c1, t1 = e.replicate_tick_export(lp)
        of = o.replicate_tick(lp)
        oc, ot = o.export_group_status(lp)
        assert np.array_equal(f1, of) and np.array_equal(c1, oc) and np.array_equal(t1, ot)
        assert_states_equal(e.store_state(), o.state(), G, P, L, "sharded host tick")
        e.set_tick_shards(1)
        assert np.array_equal(e.replicate_tick(lp), o.replicate_tick(lp))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "tick after shards reset")
