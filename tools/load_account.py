"""Where the config #3 tick's HBM reads exceed the algorithmic words
(the overfetch account): the oracle's algorithmic bitmaps
(ora_count_bits) are OR-ed with the log words k_tick_group<5> loads beyond
them — read from the kernel's indexing in mraft_tick.hip / mraft_pass.h, not
measured — and the union is rounded to lines. Two load patterns over-read:

* compare chunks: pass_pipe loads a follower's terms 256 Indexes at a time
  (chunks start on the 128-B line of the leader's row that holds plo, the
  group's lowest compared Index), so a merge whose first mismatch m falls
  inside a chunk has read the chunk's words past m (up to cend);
* ConflictIndex probes: one 64-term load below prev per scanning follower
  ([max(prev-64, dummy+2), prev-1]), then 64-term windows further down,
  however short the run of equal terms is.

Also: the lines of the header's single-word log reads that the pass streams
again (a second fetch when L2 has dropped them in between).

Prints the line-granular reads (32 / 64 / 128 B) of the algorithmic words
alone and with each pattern added, beside the PMC reads
(profiles/pmc_traffic_s2.json).

Usage: python tools/load_account.py [out.json]   (CPU, a few minutes, ~20 GB)"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from multiraft_amd import synth_seed, synth_tick_state  # noqa: E402
from oracle_lib import Oracle, lib  # noqa: E402

G, P, L = 65536, 5, 4096
A_LOG, A_COUNT = 8, 12
LEADER = 1  # MRAFT_LEADER


def words_of(lo, hi):
    """Concatenated [lo_i, hi_i) ranges (int64) and the owner index of each."""
    n = np.maximum(hi - lo, 0)
    own = np.repeat(np.arange(len(lo)), n)
    off = np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n)
    return lo[own] + off, own


def main():
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=8)
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    log = st["log_term"].reshape(-1)
    head, dummy, last = st["log_head"], st["dummy_index"], st["last_index"]
    term, role = st["current_term"], st["state"]
    nxt = st["next_index"].reshape(-1, P)

    def pos(slot, idx):
        return slot.astype(np.int64) * L + (head[slot] + idx - dummy[slot]) % L

    # the algorithmic bitmaps
    o = Oracle(G, P, L, st)
    ol = lib()
    ol.ora_count_bits.restype = ctypes.POINTER(ctypes.c_uint64)
    ol.ora_count_bits.argtypes = [ctypes.c_int32]
    ol.ora_count_base.restype = ctypes.c_int64
    ol.ora_count_base.argtypes = [ctypes.c_int32]
    ol.ora_count_enable(ctypes.byref(o._e))
    try:
        o.replicate_tick(lp)
        base = [int(ol.ora_count_base(a)) for a in range(A_COUNT + 1)]
        nw = (base[A_COUNT] + 63) // 64
        bits = np.ctypeslib.as_array(ol.ora_count_bits(0), shape=(nw,)).copy()
    finally:
        ol.ora_count_disable()
    del o
    allbits = np.unpackbits(bits.view(np.uint8), bitorder="little").astype(bool)
    del bits
    alg_log = allbits[base[A_LOG]:base[A_LOG + 1]].copy()
    other = {lw: sum(int(np.add.reduceat(allbits[base[a]:base[a + 1]],
                                         np.arange(0, base[a + 1] - base[a], lw)).astype(bool).sum())
                     for a in range(A_COUNT) if a != A_LOG) for lw in (8, 16, 32)}
    del allbits

    # the tick's AppendEntries items: every follower of every leader whose prev lies in the log
    g = np.arange(G)
    ld = g * P + lp
    isl = (lp >= 0) & (role[np.maximum(ld, 0)] == LEADER)
    gl, ldl = g[isl], ld[isl]
    items_g, items_p = [], []
    for p in range(P):
        sel = lp[gl] != p
        items_g.append(gl[sel]); items_p.append(np.full(int(sel.sum()), p))
    ig, ip = np.concatenate(items_g), np.concatenate(items_p)
    il = ig * P + lp[ig]
    f = ig * P + ip
    prev = nxt[il, ip].astype(np.int64) - 1
    ae = (prev >= dummy[il]) & (prev <= last[il])
    ig, ip, il, f, prev = ig[ae], ip[ae], il[ae], f[ae], prev[ae]
    T = term[il]
    fd, fl = dummy[f].astype(np.int64), last[f].astype(np.int64)
    stale = T < term[f]
    ok = ~stale & (prev >= fd)
    inside = ok & (prev <= fl)
    plt = log[pos(il, prev)]
    fpt = np.where(inside, log[pos(f, np.clip(prev, fd, fl))], 0)
    succ = inside & (fpt == plt)
    merge = succ
    miss = ok & ~succ

    # compare chunks
    mi = np.nonzero(merge)[0]
    start = prev[mi] + 1
    cend = np.minimum(last[il[mi]], fl[mi]) + 1
    m = cend.copy()
    for a in range(0, len(mi), 4096):
        sl = slice(a, a + 4096)
        k = int((cend[sl] - start[sl]).max(initial=0))
        if k <= 0:
            continue
        idx = start[sl][:, None] + np.arange(k)[None, :]
        valid = idx < cend[sl][:, None]
        idxc = np.where(valid, idx, start[sl][:, None])
        bad = valid & (log[pos(il[mi[sl]][:, None], idxc)] != log[pos(f[mi[sl]][:, None], idxc)])
        hit = bad.any(axis=1)
        m[sl] = np.where(hit, start[sl] + bad.argmax(axis=1), cend[sl])
    plo = np.full(G, np.iinfo(np.int64).max)
    np.minimum.at(plo, ig[mi], start)
    lb = (head[il[mi]] - dummy[il[mi]]).astype(np.int64)
    gp = plo[ig[mi]]
    c0 = gp - (((gp + lb) % L) & 31)
    cend_chunk = c0 + 256 * ((m - c0) // 256 + 1)
    over_lo = m + 1
    over_hi = np.where(m < cend, np.minimum(cend, cend_chunk), m + 1)
    w, own = words_of(over_lo, over_hi)
    cmp_words = pos(f[mi][own], w)

    # ConflictIndex probes and windows
    si = np.nonzero(miss & inside & (prev > fd + 1))[0]
    sa = fpt[si]
    lo = fd[si] + 2
    hi = prev[si] - 1
    # first Index below prev whose term differs (the scan's end), lo - 1 if none
    r = np.full(len(si), -1, np.int64)
    probe_lo = np.maximum(prev[si] - 64, lo)
    todo = np.arange(len(si))
    cur_lo, cur_hi = probe_lo.copy(), hi.copy()
    while len(todo):      # the probe window, then 64-term windows down to lo
        k = int((cur_hi[todo] - cur_lo[todo] + 1).max(initial=1))
        idx = cur_hi[todo][:, None] - np.arange(k)[None, :]
        valid = idx >= cur_lo[todo][:, None]
        t = log[pos(f[si[todo]][:, None], np.where(valid, idx, cur_lo[todo][:, None]))]
        d = valid & (t != sa[todo][:, None])
        found = d.any(axis=1)
        r[todo[found]] = idx[found, d[found].argmax(axis=1)]
        todo = todo[~found]
        todo = todo[cur_lo[todo] - 1 >= lo[todo]]
        cur_hi[todo] = cur_lo[todo] - 1
        cur_lo[todo] = np.maximum(cur_hi[todo] - 63, lo[todo])
    # simpler: each follower's scanned range is [r_or_lo, hi], rounded down to its window
    rr = np.where(r >= 0, r, lo)
    wl = np.where(rr >= probe_lo, probe_lo, np.maximum(lo, probe_lo - 64 * ((probe_lo - rr + 63) // 64)))
    w1, o1 = words_of(wl, hi + 1)
    scan_words = pos(f[si][o1], w1)

    # header single-word reads (leader log[prev] of every item, follower
    # log[prev] inside its log, the leader's log[last]) whose lines the pass
    # streams again later: fetched twice when L2 drops them in between
    hdr = np.concatenate([pos(il, prev), pos(f[inside], prev[inside]), pos(ldl, last[ldl].astype(np.int64))])
    gm = np.unique(ig[mi])
    lsl = gm * P + lp[gm]
    w_l, o_l = words_of(plo[gm], last[lsl].astype(np.int64) + 1)
    e_f = np.where(m < cend, np.minimum(cend, cend_chunk), cend)
    w_f, o_f = words_of(start, e_f)
    pass_words = np.concatenate([pos(lsl[o_l], w_l), pos(f[mi][o_f], w_f), scan_words])
    header_lines = {}
    for lw in (8, 16, 32):
        hl = np.unique(hdr // lw)
        header_lines[str(4 * lw)] = {"header_line_bytes": 4 * lw * len(hl),
                                     "also_streamed_by_the_pass": 4 * lw * len(np.intersect1d(hl, np.unique(pass_words // lw)))}
    del pass_words

    def lines(extra, lw):
        b = alg_log.copy()
        for e in extra:
            b[e] = True
        return int(b.reshape(-1, lw).any(axis=1).sum()) + other[lw]

    out = {"workload": "config #3 tick (65,536 groups x 5 peers x 4,096)",
           "items": int(len(f)), "merges": int(len(mi)),
           "merges_with_mismatch": int((m < cend).sum()),
           "compare_overread_words": int(len(cmp_words)),
           "scans": int(len(si)), "scan_words_loaded": int(len(scan_words)),
           "header_lines": header_lines, "lines": {}}
    for lw in (8, 16, 32):
        a = lines([], lw)
        c = lines([cmp_words], lw)
        s_ = lines([scan_words], lw)
        cs = lines([cmp_words, scan_words], lw)
        out["lines"][str(4 * lw)] = {"algorithmic_read_bytes": 4 * lw * a,
                                     "with_compare_chunks": 4 * lw * c,
                                     "with_conflict_probes": 4 * lw * s_,
                                     "with_both": 4 * lw * cs}
    pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_s2.json")))
    out["pmc_read_bytes"] = pmc["hbm_read_bytes_per_dispatch"] * pmc["launches_per_step"]
    out["pmc_tag"] = pmc["tag"]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
