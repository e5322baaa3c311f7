"""Message-level batch builders shared by the CPU and GPU parity tests: the
gather -> handle -> fold path a host drives for network-delivered batches
(include/mraft.h; raft_append_entry.go:20-162)."""
import numpy as np

from multiraft_amd._abi import AE_ARGS, AE_RESULT, LEADER
from multiraft_amd.engine import entry_positions


def all_follower_items(lp, G, P):
    """(leader slot, peer) for every follower of every group with a leader."""
    g = np.repeat(np.arange(G), P - 1)
    ld = g * P + np.repeat(lp, P - 1)
    q = np.tile(np.arange(P - 1), G)
    peers = np.where(q < np.repeat(lp, P - 1), q, q + 1)
    keep = np.repeat(lp >= 0, P - 1)
    return ld[keep].astype(np.int32), peers[keep].astype(np.int32)


def external_entries(args, ok, st, L, misalign=True):
    """Copy every gathered item's entries (a view into the leader's log ring,
    entries_offset: a logical ring position, unrolled through log_head by
    multiraft_amd.entry_positions) into one external buffer, as the network
    would deliver them; item j starts at a 16-B aligned position plus (j % 4)
    words when `misalign`. Returns (args with rebased entries_offset, buffer)."""
    a2 = args.copy()
    n = np.where(ok, args["n_entries"], 0).astype(np.int64)
    pad = (np.arange(len(args)) % 4) if misalign else np.zeros(len(args), np.int64)
    span = ((n + 3) // 4) * 4 + 4                      # each item in its own 16-B aligned slab
    start = np.concatenate([[0], np.cumsum(span)[:-1]]) + pad
    total = int(span.sum()) + 4
    buf = np.zeros(total, np.int32)
    idx_item = np.repeat(np.arange(len(args)), n)
    within = np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n)
    dst = start[idx_item] + within
    buf[dst] = st["log_term"][entry_positions(st["log_head"], L, args["entries_offset"], n)]
    a2["entries_offset"] = np.where(ok, start, 0)
    return a2, buf


def results_of(slots, peers, args, rep, herr, G, P):
    """AE_RESULT records for the replies of the handled items, one segment per
    leader slot (ascending slot, peer order kept), and the segment boundaries."""
    ok = herr == 0
    res = np.zeros(int(ok.sum()), dtype=AE_RESULT)
    res["slot"], res["peer"] = slots[ok], peers[ok]
    res["args_term"], res["args_prev_log_index"] = args["term"][ok], args["prev_log_index"][ok]
    res["args_n_entries"] = args["n_entries"][ok]
    res["reply_term"], res["reply_success"] = rep["term"][ok], rep["success"][ok]
    res["reply_conflict_index"] = rep["conflict_index"][ok]
    order = np.argsort(res["slot"], kind="stable")
    res = res[order]
    cut = np.nonzero(np.diff(res["slot"]))[0] + 1
    seg = np.concatenate([[0], cut, [len(res)]]).astype(np.int64)
    return res, seg


def stale_second_leader_state(st, lp, G, P, L, rng, groups):
    """Make a second, stale leader in each of `groups`: replica q != lp[g]
    becomes Leader one term below the real leader, with a log that diverges
    from the real leader's after index d and nextIndex pointing into it. The
    batch [lp -> q, q -> r] then has q's row both written (by the first item)
    and read as entries (by the second)."""
    st = {k: v.copy() for k, v in st.items()}
    pairs = []
    for g in groups:
        l = int(lp[g])
        q = (l + 1) % P
        r = (l + 2) % P
        ls, qs = g * P + l, g * P + q
        T = int(st["current_term"][ls])
        st["state"][qs] = LEADER
        st["current_term"][qs] = max(1, T - 1)
        st["dummy_index"][qs] = 0
        llast = int(st["last_index"][ls])
        qlast = min(L - 1, max(4, llast))
        lrow = st["log_term"][ls * L:(ls + 1) * L]
        qrow = st["log_term"][qs * L:(qs + 1) * L]
        d = int(rng.integers(1, max(2, min(qlast, llast) - 1)))
        lrow[d + 1:llast + 1] = T             # the real leader's entries past d: its own term
        qrow[:d + 1] = lrow[:d + 1]
        qrow[d + 1:qlast + 1] = max(1, T - 1)  # q's diverging tail
        st["last_index"][qs] = qlast
        st["commit_index"][qs] = min(int(st["commit_index"][qs]), d)
        st["last_applied"][qs] = min(int(st["last_applied"][qs]), int(st["commit_index"][qs]))
        # the real leader's view of q: probe at a point inside the common prefix
        st["next_index"][ls * P + q] = int(rng.integers(1, d + 1))
        # the stale leader's view of r
        st["next_index"][qs * P + r] = int(rng.integers(1, qlast + 1))
        pairs.append((ls, q))
        pairs.append((qs, r))
    slots = np.array([s for s, _ in pairs], np.int32)
    peers = np.array([p for _, p in pairs], np.int32)
    return st, slots, peers


def stale_cycle_state(st, lp, G, P, L, rng, groups, k):
    """Stale leaders sending to each other in a ring: in each of `groups`,
    replicas r_0 = lp[g], r_1, ..., r_{k-1} (k <= P) are all Leaders, r_j one
    term below r_{j-1} with a log that diverges from r_{j-1}'s, and the batch
    holds r_j -> r_{j+1 mod k}. Every item then reads a row another item
    writes and writes a row another item reads: a cycle of k deferred items
    whose entries the engine must take as they were before the call (staged,
    or, past the stage capacity, one of them copied to break the cycle).
    2 <= k <= P."""
    st = {kk: v.copy() for kk, v in st.items()}
    pairs = []
    for g in groups:
        l = int(lp[g])
        rs = [(l + j) % P for j in range(k)]
        slots = [g * P + r for r in rs]
        T = int(st["current_term"][slots[0]])
        prev_row = st["log_term"][slots[0] * L:(slots[0] + 1) * L]
        prev_last = int(st["last_index"][slots[0]])
        for j in range(1, k):
            s = slots[j]
            st["state"][s] = LEADER
            st["current_term"][s] = max(1, T - j)
            st["dummy_index"][s] = 0
            last = min(L - 1, max(4, prev_last))
            row = st["log_term"][s * L:(s + 1) * L]
            d = int(rng.integers(1, max(2, min(last, prev_last) - 1)))
            row[:d + 1] = prev_row[:d + 1]
            row[d + 1:last + 1] = max(1, T - j)
            st["last_index"][s] = last
            st["commit_index"][s] = min(int(st["commit_index"][s]), d)
            st["last_applied"][s] = min(int(st["last_applied"][s]), int(st["commit_index"][s]))
            prev_row, prev_last = row, last
        for j in range(k):
            a, b = slots[j], slots[(j + 1) % k]
            st["next_index"][a * P + (b % P)] = int(rng.integers(1, int(st["last_index"][a]) + 2))
            pairs.append((a, b % P))
    return st, np.array([a for a, _ in pairs], np.int32), np.array([b for _, b in pairs], np.int32)


def shift_indices(st, off):
    """The same logs with every Raft Index moved up by `off` (terms, rings and
    every relation between Indexes unchanged): dummy, last, commit, lastApplied,
    matchIndex and nextIndex. Raft's decisions depend on Index differences
    only, so a step on the shifted state equals the step on the original with
    its Index outputs shifted (the Index-domain invariance tests)."""
    st = {k: v.copy() for k, v in st.items()}
    for k in ("dummy_index", "last_index", "commit_index", "last_applied", "match_index", "next_index"):
        st[k] = (st[k].astype(np.int64) + off).astype(np.int32)
    return st


def top_offset(st, j=0):
    """The shift that puts the highest Index of `st` (its last, or a
    nextIndex - 1) at 2^31 - 2 - j: the top of the engine's Index domain
    (include/mraft.h: nextIndex = Index + 1 must be an int32)."""
    hi = max(int(st["last_index"].max()), int(st["next_index"].max()) - 1)
    return (2**31 - 2 - j) - hi


def deferred_graph_state(G, P, L, rng, c=None):
    """Every replica a follower at term 5 with one common log prefix
    (Index 0 .. c) and its own suffix of non-decreasing terms up to a random
    last Index: an AppendEntries at prev = c (prevLogTerm = the prefix's term)
    from ANY replica's row matches at every receiver and merges that row's
    suffix — real writes, whatever rows the batch wires together."""
    n = G * P
    c = c if c is not None else L // 4
    st = {k: np.zeros(n, np.int32) for k in ("current_term", "voted_for", "state", "commit_index", "last_applied",
                                            "dummy_index", "last_index", "granted_votes", "persist_dirty",
                                            "log_head", "has_snapshot", "terms_sorted")}
    st["current_term"][:] = 5
    st["voted_for"][:] = -1
    st["state"][:] = 3  # Follower
    st["last_index"][:] = rng.integers(c + 1, L, size=n)
    st["commit_index"][:] = rng.integers(0, c + 1, size=n)
    st["last_applied"][:] = st["commit_index"]
    st["terms_sorted"][:] = 1
    st["match_index"] = np.zeros(n * P, np.int32)
    st["next_index"] = np.zeros(n * P, np.int32)
    log = np.zeros((n, L), np.int32)
    prefix = np.sort(rng.integers(1, 3, size=c + 1)).astype(np.int32)
    prefix[0] = 0
    log[:, :c + 1] = prefix
    for s in range(n):
        last = int(st["last_index"][s])
        log[s, c + 1:last + 1] = np.sort(rng.integers(3, 6, size=last - c))
    st["log_term"] = log.reshape(-1)
    return st, c


def deferred_graph_batch(st, G, P, L, c, rng, n_items, long_cycle=0, self_refs=0):
    """n_items AppendEntries by reference at distinct receiving slots, each
    reading the suffix of a random replica's row (entries_offset = that row,
    Index c+1 on): the rows read and written form a random functional graph —
    trees, chains and cycles of deferred items (an item whose slot another
    item reads is deferred; one whose source row another item writes is
    staged). Optionally one explicit cycle of `long_cycle` items (longer than
    the fallback's walk) and `self_refs` items reading their own row."""
    n = G * P
    recv = rng.permutation(n)[:n_items]
    src = rng.integers(0, n, size=n_items)
    # sources mostly among the receivers: many deferred items
    among = rng.random(n_items) < 0.8
    src[among] = recv[rng.integers(0, n_items, size=int(among.sum()))]
    if long_cycle:
        k = long_cycle
        src[:k] = np.roll(recv[:k], -1)   # item j reads the row item j+1 writes: one k-cycle
    if self_refs:
        src[k if long_cycle else 0:][:self_refs] = recv[k if long_cycle else 0:][:self_refs]
    a = np.zeros(n_items, dtype=AE_ARGS)
    a["slot"] = recv
    a["term"] = 9
    a["leader_id"] = (recv + 1) % P
    a["prev_log_index"] = c
    a["prev_log_term"] = st["log_term"].reshape(n, L)[0, c]
    a["n_entries"] = st["last_index"][src] - c
    a["leader_commit"] = c
    a["flags"] = 1
    a["entries_offset"] = src.astype(np.int64) * L + (c + 1)
    return a
