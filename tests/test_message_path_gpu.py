"""Message-level parity on the GPU (the entry points a host calls for
network-delivered batches, include/mraft.h): gather (a3,
raft_append_entry.go:20-54) -> HandleAppendEntries (a4, :108-162) ->
processAppendEntriesReply + advanceCommitIndexForLeader (a2 + a1, :66-105),
against the CPU oracle, bit for bit: replies, error codes, flags and the full
state — at BASELINE config #3 size, with external entry buffers at aligned and
misaligned offsets and tails of thousands of entries, and with entries by
reference into the engine's own log, including batches that rewrite a row
another of their items reads."""
import numpy as np
import pytest

from index_domain_cases import MSG_MODES, message_case
from message_cases import all_follower_items, external_entries, results_of, stale_second_leader_state
from oracle_lib import Oracle, assert_states_equal

from multiraft_amd import Engine, synth_seed, synth_tick_state

pytestmark = pytest.mark.gpu


def _big_equal(a, b, G, P, L, ctx, rows=8192):
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


def _message_round(e, o, st, slots, peers, G, P, L, mode, equal):
    args, gerr = e.gather_append_args(slots, peers)
    oargs, ogerr = o.gather_append_args(slots, peers)
    assert np.array_equal(gerr, ogerr) and np.array_equal(args, oargs)
    ok = gerr == 0
    if mode == "reference":
        rep, herr, gres = e.handle_append_entries(args, None, results=True)
        orep, oherr = o.handle_append_entries(args, None)
    else:
        a2, buf = external_entries(args, ok, st, L, misalign=(mode == "misaligned"))
        a2 = a2[ok]
        rep, herr, gres = e.handle_append_entries(a2, buf, results=True)
        orep, oherr = o.handle_append_entries(a2, buf)
        args, slots, peers = args[ok], slots[ok], peers[ok]
    assert np.array_equal(herr, oherr), f"{mode}: handle errors"
    assert np.array_equal(rep, orep), f"{mode}: replies"
    equal(e.store_state(), o.state(), G, P, L, f"{mode}: after handle")
    res, seg = results_of(slots, peers, args, rep, herr, G, P)
    # the handler's own reply records (mraft_handle_append_entries_ex) are the
    # host-assembled ones, item by item; failed items carry slot -1
    okh = herr == 0
    hand = gres[okh][np.argsort(gres["slot"][okh], kind="stable")]
    assert np.array_equal(hand, res), f"{mode}: handler's reply records"
    assert (gres["slot"][~okh] == -1).all()
    f, ferr = e.process_append_replies(res, seg)
    of, oferr = o.process_append_replies(res, seg)
    assert np.array_equal(ferr, oferr) and np.array_equal(f, of), f"{mode}: fold"
    equal(e.store_state(), o.state(), G, P, L, f"{mode}: after fold")
    return rep, herr


@pytest.mark.parametrize("mode", ["aligned", "misaligned", "reference"])
def test_message_path_full_config3_gpu(mode):
    """65,536 groups x 5 peers x 4,096-entry logs (the bench workload): all
    262,144 AppendEntries of one round through gather -> handle -> fold."""
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    slots, peers = all_follower_items(lp, G, P)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        rep, herr = _message_round(e, o, st, slots, peers, G, P, L, mode, _big_equal)
        n_ent = e.gather_append_args(slots, peers)[0]["n_entries"]
    # the round exercised long tails and every outcome
    assert int(n_ent.max()) > 3000
    assert (rep["success"] == 1).sum() > 50000 and (rep["success"] == 0).sum() > 50000


@pytest.mark.parametrize("mode", ["aligned", "misaligned", "reference"])
def test_handle_long_batches_gpu(mode):
    """Thousand-entry tails into full-size rows at a small G (the pipelined
    copy loop over an external buffer runs many iterations; uneven ends)."""
    G, P, L = 96, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=123)
    slots, peers = all_follower_items(lp, G, P)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        _message_round(e, o, st, slots, peers, G, P, L, mode, assert_states_equal)


def test_stale_second_leader_by_reference_gpu():
    """Entries by reference (entry_terms NULL) in a batch that rewrites a row
    another of its items reads (lp -> q and q -> r, q a stale leader): the
    engine stages those entries as the reference's gather-time copy would."""
    G, P, L = 256, 5, 128
    rng = np.random.default_rng(17)
    st, lp, _ = synth_tick_state(G, P, L, seed=92)
    st, slots, peers = stale_second_leader_state(st, lp, G, P, L, rng, range(0, G, 2))
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        _message_round(e, o, st, slots, peers, G, P, L, "reference", assert_states_equal)


def _cross_group_runs(args, ok, G, P, rng, run):
    """By-reference messages whose entries are shared by long runs: each
    gathered message is repeated `run` times, each copy addressed to a distinct
    receiving slot of another group (longer than a set: the plan must split
    the run), the batch then interleaved with messages of other sources."""
    a = args[ok]
    used = set(a["slot"].tolist())
    free = [s for s in rng.permutation(G * P).tolist() if s not in used]
    out = []
    for k in range(0, len(a), 5):
        for j in range(run):
            if not free:
                break
            m = a[k].copy()
            m["slot"] = free.pop()
            out.append(m)
    return np.array(out, dtype=args.dtype)


@pytest.mark.parametrize("order", ["gathered", "shuffled", "long_runs", "with_errors"])
def test_handle_sets_gpu(order):
    """Message sets (messages reading the same entries, one wave each) in
    every arrangement the plan must cut correctly: the gather's own order
    (one set per leader), shuffled (sets of one), runs longer than a set,
    and runs broken by duplicate-slot and malformed messages."""
    G, P, L = 512, 5, 256
    rng = np.random.default_rng(7 + len(order))
    st, lp, _ = synth_tick_state(G, P, L, seed=303)
    slots, peers = all_follower_items(lp, G, P)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        args, gerr = e.gather_append_args(slots, peers)
        ok = gerr == 0
        if order == "gathered":
            batch = args[ok]
        elif order == "shuffled":
            batch = args[ok][rng.permutation(int(ok.sum()))]
        elif order == "long_runs":
            batch = _cross_group_runs(args, ok, G, P, rng, 11)
        else:
            batch = args[ok].copy()
            dup = rng.choice(len(batch), len(batch) // 9, replace=False)
            for j in dup:
                batch[j]["slot"] = batch[(j + 2) % len(batch)]["slot"]   # a duplicate receiving slot
            bad = rng.choice(len(batch), len(batch) // 13, replace=False)
            batch["entries_offset"][bad] = -5                              # malformed reference
            zero = rng.choice(len(batch), len(batch) // 11, replace=False)
            batch["n_entries"][zero] = 0
        rep, herr = e.handle_append_entries(batch, None)
        orep, oherr = o.handle_append_entries(batch, None)
        assert np.array_equal(herr, oherr)
        assert np.array_equal(rep, orep)
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"sets ({order})")
        if order == "with_errors":
            assert (herr != 0).any() and (herr == 0).any()


@pytest.mark.parametrize("j", [0, 7])
@pytest.mark.parametrize("mode", MSG_MODES)
def test_handle_high_indices_gpu(mode, j):
    """The highest Index at 2^31 - 2 - j (the top of the engine's domain,
    include/mraft.h), prevLogIndex far above 2^30: entries from a host buffer
    (aligned / misaligned), by reference in place, deferred in place, staged,
    and in the ordered fallback (stage capacity 0 and 64), with the
    sorted-terms flag set — GPU == oracle through gather, handle and fold
    (tests/index_domain_cases.py; the flat-source read that faulted in round
    5, DESIGN.md §5 r5_v1, runs on every one of these)."""
    assert message_case(mode, j) > 0


@pytest.mark.parametrize("S", [2, 3])
def test_message_path_shard_pipelines_gpu(S):
    """The bench's message path as S shard pipelines (bench.message_path: an
    engine on a dedicated queue per contiguous group range, bound to SoA
    slices of one state image, one host thread each) leaves the same state as
    the oracle running gather -> HandleAppendEntries -> the reply fold over
    the whole batch (the groups share nothing, raft.go:16-40)."""
    import torch

    import bench
    from multiraft_amd import synth_seed
    G, P, L = 768, 5, 256
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3) + S)
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    copies = [{k: v.clone() for k, v in master.items()} for _ in range(2)]
    bench.message_path(master, copies, lp, G, P, L, dev, S, 1)
    got = {k: v.cpu().numpy() for k, v in copies[0].items()}
    o = Oracle(G, P, L, st)
    slots, peers = all_follower_items(lp, G, P)
    args, gerr = o.gather_append_args(slots, peers)
    assert (gerr == 0).all()
    rep, herr = o.handle_append_entries(args, None)
    res, seg = results_of(slots, peers, args, rep, herr, G, P)
    o.process_append_replies(res, seg)
    assert_states_equal(got, o.state(), G, P, L, f"{S} pipelines")
