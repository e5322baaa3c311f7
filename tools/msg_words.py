"""Algorithmic HBM words of one HandleAppendEntries batch by reference
(k_handle_set), from the state before the call and the
replies: what the handler must read and write, whatever kernel runs it.

Per message: its args record (10 words) and its set-head byte (1/4 word,
round 5; rounds 2-4 read a plan word pair, 2) read, its reply (4) written; the receiving follower's term, dummy, last, commit and
ring head (5) read; log[prev] (1) when prev lies inside the follower's log;
the ConflictIndex scan's words; for a merge, the follower's terms compared up
to the first mismatch and the entries written from there; the state words a
follower's reply changes (role; term and votedFor on adoption; last on
truncation; terms_sorted when an append changes it (include/mraft.h); commit
when it moves; the persist-flag read-modify-write).
Per set (messages reading the same entries): the shared entries once, from
the lowest compared Index to the highest one any message of the set needs
(round 5: no set record; rounds 2-4 read one, 2 words).
raft_append_entry.go:108-162, raft_log.go:92-96."""
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
    words = len(args) * (10 + 4) + len(args) / 4 + int(ok.sum()) * 5 + int(inside.sum())
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
    # state written by the replies (:111-161)
    wr = ok & ~stale
    adopt = wr & (args["term"] > ft)
    words += int(wr.sum()) + 2 * int(adopt.sum()) + 2 * int((stale | wr).sum())
    newlast = np.zeros(len(args), bool)
    newlast[mi[copies]] = True
    words += int(newlast.sum())
    # terms_sorted after an append from Index m: cleared without the args'
    # flag, set with it when m - 1 is the dummy (k_handle_set)
    flag = (args["flags"][mi] & 1) != 0
    words += int((copies & (~flag | (m == fd[mi] + 1))).sum())
    last_after = np.where(newlast, prev + n, fl)
    words += int((merge & (args["leader_commit"] > fc) & (np.minimum(args["leader_commit"], last_after) >= 0)).sum())
    return {"words": words, "sets": n_sets, "merges": int(merge.sum()), "copied": int(np.where(copies, phi - m + 1, 0).sum())}


def _quorum(m, me, P):
    """h-th largest (h = P/2) of matchIndex[j != me] (raft_append_entry.go:91-98)."""
    v = sorted((m[j] for j in range(P) if j != me), reverse=True)
    return v[P // 2 - 1] if P // 2 >= 1 else max(v)


def fold_words(st, res, seg, P, L):
    """Algorithmic HBM words of one processAppendEntriesReply +
    advanceCommitIndexForLeader batch (k_fold; raft_append_entry.go:66-105)
    from the state before the call and the reply records, whatever kernel
    runs it. Per reply: its record (8 words) read, its flag and error word
    written. Per segment (one leader replica): the segment bounds (int64),
    the replica's term, role, commit, last, dummy, ring head and
    terms_sorted; nextIndex of every replying peer (the gate, :73-74);
    matchIndex of every peer but the leader's when a1 runs (:91-97); a1's log
    words: for each evaluation (:78) the term of min(M*, last) and, unless it
    settles the evaluation (it equals currentTerm, or the replica's terms are
    sorted and it is below currentTerm: include/mraft.h), the terms below it
    down to the first one equal to currentTerm, or to the highest Index an
    earlier evaluation of the segment examined (each word read once per
    segment); written: nextIndex (and matchIndex on
    success) of every reply that passes the gate, commitIndex when it moves,
    term / role / votedFor and the persist flag on a step-down.
    Returns {"words", "a1_log_words", "segments", "evaluations"}."""
    log = st["log_term"].reshape(-1)
    head, dummy, last = st["log_head"], st["dummy_index"], st["last_index"]
    term, role, commit = st["current_term"], st["state"], st["commit_index"]
    srt = st["terms_sorted"]
    match = st["match_index"].reshape(-1, P)
    nxt = st["next_index"].reshape(-1, P)
    n_seg = len(seg) - 1
    words = 10 * len(res) + 2 * (n_seg + 1)
    a1w = evals = 0
    commits = commit.copy()                      # the commitIndex the fold leaves (self-check)
    for sg in range(n_seg):
        b, e = int(seg[sg]), int(seg[sg + 1])
        if b >= e:
            continue
        s = int(res["slot"][b])
        me = s % P
        T, r, c = int(term[s]), int(role[s]), int(commit[s])
        lst, d, h = int(last[s]), int(dummy[s]), int(head[s])
        m, nx = [int(x) for x in match[s]], [int(x) for x in nxt[s]]
        words += 7 + len(set(int(x) for x in res["peer"][b:e]))
        t, H, a1 = T, c, False
        wrote = 0
        for i in range(b, e):
            pr, rt = int(res["peer"][i]), int(res["reply_term"][i])
            at, ap = int(res["args_term"][i]), int(res["args_prev_log_index"][i])
            if rt > t:                                            # :67-72
                t, r = rt, 3
                wrote |= 1
            elif rt == t and r == 1 and at == t and ap == nx[pr] - 1:   # :73-74
                if int(res["reply_success"][i]):
                    mv = int(res["args_n_entries"][i]) + ap
                    m[pr], nx[pr] = mv, mv + 1
                    words += 2
                    a1 = True
                    evals += 1
                    top = min(_quorum(m, me, P), lst)
                    if top > H:                                   # a1: (H, top], currentTerm = T here
                        tt = int(log[s * L + (h + top - d) % L])
                        if tt != T and srt[s] and tt < T:          # settled by the top term
                            k = H
                            a1w += 1
                        else:
                            idx = np.arange(H + 1, top + 1)
                            hit = np.nonzero(log[s * L + (h + idx - d) % L] == T)[0]
                            k = int(idx[hit[-1]]) if len(hit) else H
                            a1w += top - max(k, H + 1) + 1
                        if k > H:
                            c = k
                        H = top
                else:
                    nx[pr] = int(res["reply_conflict_index"][i])
                    words += 1
        if a1:
            words += P - 1
        if c != int(commit[s]):
            words += 1
        if wrote:
            words += 4
        commits[s] = c
    return {"words": words + a1w, "a1_log_words": a1w, "segments": n_seg, "evaluations": evals,
            "commit": commits}
