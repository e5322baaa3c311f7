"""CPU side of the deferred-item graphs (tests/message_cases.py
deferred_graph_batch): the batches really are what the GPU tests need —
many deferred items, chains, short and long cycles, self-references — and
the oracle handles them as the reference's gather-time copy says
(src/raft/raft_append_entry.go:50-54: every item reads its source as it was
before the call)."""
import numpy as np

from message_cases import deferred_graph_batch, deferred_graph_state
from oracle_lib import Oracle


def _graph_stats(a, G, P, L):
    n = len(a)
    recv = a["slot"].astype(np.int64)
    src = a["entries_offset"] // L
    owner = {int(r): i for i, r in enumerate(recv)}
    writer = np.array([owner.get(int(s), -1) for s in src])
    deferred = np.isin(recv, src)
    cyc = 0
    seen = set()
    longest = 0
    for i in range(n):
        if i in seen or not deferred[i]:
            continue
        path, x = [], i
        while x >= 0 and x not in path and x not in seen:
            path.append(x)
            x = writer[x]
        if x >= 0 and x in path:
            cyc += 1
            longest = max(longest, len(path) - path.index(x))
        seen.update(path)
    return int(deferred.sum()), cyc, longest


def test_graph_batches_have_the_shapes():
    rng = np.random.default_rng(600)
    G, P, L = 64, 5, 64
    st, c = deferred_graph_state(G, P, L, rng)
    a = deferred_graph_batch(st, G, P, L, c, rng, 200, long_cycle=40, self_refs=3)
    nd, cycles, longest = _graph_stats(a, G, P, L)
    assert nd > 100 and cycles >= 2 and longest == 40
    o = Oracle(G, P, L, st)
    rep, err = o.handle_append_entries(a, None)
    assert (err == 0).all() and (rep["success"] == 1).all()
    # the receivers' rows now hold their sources' suffixes as they were before the call
    log0 = st["log_term"].reshape(G * P, L)
    log1 = o.state()["log_term"].reshape(G * P, L)
    src = a["entries_offset"] // L
    for r, s_ in zip(a["slot"], src):
        assert np.array_equal(log1[r, c + 1:st["last_index"][s_] + 1], log0[s_, c + 1:st["last_index"][s_] + 1])


def test_bench_deferred_batches_shape():
    """bench.py's deferred-heavy config #3 batches (secondary.message_path_deferred),
    at a small size: every gather succeeds, every stale leader's receiver is
    deferred (stale) or in a 2-cycle (cycles), and the oracle handles them."""
    import bench
    from multiraft_amd import synth_tick_state
    G, P, L = 64, 5, 128
    st, lp, _ = synth_tick_state(G, P, L, seed=710, nthreads=1)
    for kind in ("stale", "cycles"):
        st2, slots, peers = bench.deferred_batch_state(st, lp, G, P, L, kind)
        o = Oracle(G, P, L, st2)
        args, gerr = o.gather_append_args(slots, peers)
        assert (gerr == 0).all(), kind
        src = np.where(args["n_entries"] > 0, args["entries_offset"] // L, -1)
        deferred = np.isin(args["slot"], src[src >= 0])
        n_stale = int(((lp[::2]) >= 0).sum())
        assert deferred.sum() >= n_stale * (2 if kind == "cycles" else 1) - 2, kind
        rep, err = o.handle_append_entries(args, None)
        assert (err == 0).all() and (rep["success"] == 1).any(), kind
        assert len(slots) == (4 * int((lp >= 0).sum()) + (n_stale if kind == "cycles" else 0)), kind
