"""Algorithmic HBM words of one HandleAppendEntries batch by reference
(k_handle_set), from the state before the call and the
replies: what the handler must read and write, whatever kernel runs it.

Per message: its args record (10 words) and plan word pair (soff, 2) read,
its reply (4) written; the receiving follower's term, dummy, last, commit and
ring head (5) read; log[prev] (1) when prev lies inside the follower's log;
the ConflictIndex scan's words; for a merge, the follower's terms compared up
to the first mismatch and the entries written from there; the state words a
follower's reply changes (role; term and votedFor on adoption; last on
truncation; commit when it moves; the persist-flag read-modify-write).
Per set (messages reading the same entries): the shared entries once, from
the lowest compared Index to the highest one any message of the set needs,
plus the set record (2). raft_append_entry.go:108-162, raft_log.go:92-96."""
import numpy as np


def _terms(log, head, dummy, rows, idx, L):
    """Terms of Index idx (2-D, rows x k) in ring rows `rows`."""
    pos = (head[rows][:, None] + idx - dummy[rows][:, None]) % L
    return log[rows[:, None].astype(np.int64) * L + pos]


def handle_words(st, args, rep, herr, G, P, L, chunk=2048):
    log = st["log_term"].reshape(-1)
    head, dummy, last = st["log_head"], st["dummy_index"], st["last_index"]
    term, commit = st["current_term"], st["commit_index"]
    f = args["slot"].astype(np.int64)
    prev, n = args["prev_log_index"].astype(np.int64), args["n_entries"].astype(np.int64)
    src = args["entries_offset"] // L
    ok = herr == 0
    fd, fl, ft, fc = dummy[f], last[f], term[f], commit[f]
    stale = ok & (args["term"] < ft)
    below = ok & ~stale & (prev < fd)
    inside = ok & ~stale & ~below & (prev <= fl)
    words = len(args) * (10 + 2 + 4) + int(ok.sum()) * 5 + int(inside.sum())
    miss = ok & ~stale & ~below & (rep["success"] == 0)
    merge = ok & ~stale & ~below & (rep["success"] == 1)
    # ConflictIndex scan (:136-142): Indexes prev-1 down to the first other term
    scan = miss & inside & (prev > fd + 1)
    words += int(np.maximum(0, prev[scan] - rep["conflict_index"][scan].astype(np.int64) + 1).sum())
    # merges: first mismatch per message
    mi = np.nonzero(merge)[0]
    plo, phi = prev[mi] + 1, prev[mi] + n[mi]
    cend = np.minimum(phi, fl[mi]) + 1
    m = cend.copy()
    for a in range(0, len(mi), chunk):
        sl = slice(a, a + chunk)
        k = int((cend[sl] - plo[sl]).max(initial=0))
        if k <= 0:
            continue
        idx = plo[sl][:, None] + np.arange(k)[None, :]
        valid = idx < cend[sl][:, None]
        idxc = np.where(valid, idx, plo[sl][:, None])
        lt = _terms(log, head, dummy, src[mi[sl]], idxc, L)
        ftm = _terms(log, head, dummy, f[mi[sl]], idxc, L)
        bad = valid & (lt != ftm)
        hit = bad.any(axis=1)
        m[sl] = np.where(hit, plo[sl] + bad.argmax(axis=1), cend[sl])
    mismatch = m < cend
    shorter = ~mismatch & (cend < phi + 1)
    copies = mismatch | shorter
    words += int(np.where(mismatch, m - plo + 1, cend - plo).sum())         # follower terms compared
    words += int(np.where(copies, phi - m + 1, 0).sum())                     # entries written
    # entries read once per set: lowest compared Index to the highest needed
    need_hi = np.where(copies, phi, cend - 1)
    key = (src[mi] * (1 << 20) + phi) if len(mi) else np.zeros(0, np.int64)
    if len(mi):
        order = np.argsort(key, kind="stable")
        ks, lo_s, hi_s = key[order], plo[order], need_hi[order]
        cut = np.concatenate([[0], np.nonzero(np.diff(ks))[0] + 1])
        lo_set = np.minimum.reduceat(lo_s, cut)
        hi_set = np.maximum.reduceat(hi_s, cut)
        words += int(np.maximum(0, hi_set - lo_set + 1).sum())
    n_sets = len(np.unique(src[ok] * (1 << 20) + (prev[ok] + n[ok]))) if ok.any() else 0
    words += 2 * n_sets
    # state written by the replies (:111-161)
    wr = ok & ~stale
    adopt = wr & (args["term"] > ft)
    words += int(wr.sum()) + 2 * int(adopt.sum()) + 2 * int((stale | wr).sum())
    newlast = np.zeros(len(args), bool)
    newlast[mi[copies]] = True
    words += int(newlast.sum())
    last_after = np.where(newlast, prev + n, fl)
    words += int((merge & (args["leader_commit"] > fc) & (np.minimum(args["leader_commit"], last_after) >= 0)).sum())
    return {"words": words, "sets": n_sets, "merges": int(merge.sum()), "copied": int(np.where(copies, phi - m + 1, 0).sum())}
