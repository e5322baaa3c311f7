"""Adversarial random states for parity tests (test infrastructure): terms from
a tiny alphabet (accidental matches and non-monotone logs), followers sharing
random prefixes with the leader, dummies > 0, logs near the capacity L,
nextIndex below dummy (InstallSnapshot path) or beyond last (a3 panic),
commitIndex < dummyIndex (rejected), non-leader and out-of-range leader peers."""
from __future__ import annotations

import numpy as np

from multiraft_amd.engine import new_state


def random_tick_state(rng: np.random.Generator, G: int, P: int, L: int, monotone: bool = False,
                      snap: bool = False):
    """snap=True: snapshot-heavy variant — leader dummies up to L/2 and half of
    the nextIndex values at or below the leader dummy, so the fused tick's
    InstallSnapshot branch (stale, outdated, install by new log or by slice,
    dropped-on-panic) is hit in most groups."""
    st = new_state(G, P, L)
    lt = st["log_term"].reshape(G * P, L)
    lp = rng.integers(0, P, size=G).astype(np.int32)
    for g in range(G):
        ld = g * P + lp[g]
        alpha = int(rng.integers(2, 6))
        ldummy = int(rng.integers(0, 4)) if rng.random() < 0.3 else 0
        if snap:
            ldummy = int(rng.integers(0, max(2, L // 2)))
        llen = L if rng.random() < 0.3 else int(rng.integers(1, L + 1))  # slots used
        base = rng.integers(0, alpha, size=llen)
        if monotone:
            base = np.sort(base)
        lt[ld, :llen] = base
        st["dummy_index"][ld] = ldummy
        st["last_index"][ld] = ldummy + llen - 1
        lterm = int(base.max()) + int(rng.integers(0, 2))
        st["current_term"][ld] = lterm
        st["state"][ld] = 1 if rng.random() < 0.9 else int(rng.integers(2, 4))
        lastl = ldummy + llen - 1
        c = int(rng.integers(ldummy, lastl + 1))
        if rng.random() < 0.03:
            c = ldummy - 1                               # BAD_STATE
        st["commit_index"][ld] = c
        for p in range(P):
            if p == lp[g]:
                continue
            f = g * P + p
            u = rng.random()
            fd = ldummy if u < 0.7 else (int(rng.integers(0, 6)) if u < 0.85
                                         else max(0, ldummy - 1 - int(rng.integers(0, 2))))
            if snap:
                fd = int(rng.integers(0, ldummy + 3))
            # follower = leader prefix (from fd) + random tail
            share = int(rng.integers(0, max(1, lastl - fd + 2)))
            flen = min(L, max(1, share + int(rng.integers(0, 6))))
            tail = rng.integers(0, alpha, size=flen)
            if monotone:
                tail = np.sort(tail)
            row = tail.copy()
            k = min(share, flen)
            src0 = fd - ldummy
            for i in range(k):
                si = src0 + i
                if 0 <= si < llen:
                    row[i] = base[si]
            lt[f, :flen] = row
            st["dummy_index"][f] = fd
            st["last_index"][f] = fd + flen - 1
            st["current_term"][f] = max(0, lterm + int(rng.integers(-2, 2)))
            st["voted_for"][f] = int(rng.integers(-1, P))
            st["state"][f] = int(rng.integers(1, 4))
            st["commit_index"][f] = int(rng.integers(fd, fd + flen))
            if snap and rng.random() < 0.15:
                st["commit_index"][f] = fd - 1 - int(rng.integers(0, 2))   # commit < dummy
            nxt = int(rng.integers(ldummy - 1, lastl + 3)) if rng.random() < 0.1 else \
                int(rng.integers(ldummy + 1, lastl + 2))
            if snap and rng.random() < 0.5:
                nxt = int(rng.integers(max(0, ldummy - 4), ldummy + 1))
            st["next_index"][ld * P + p] = nxt
            st["match_index"][ld * P + p] = int(rng.integers(0, lastl + 2))
    st["last_applied"][:] = st["commit_index"]
    r = rng.random(G)
    lp = lp.copy()
    lp[r < 0.04] = -1
    lp[(r >= 0.04) & (r < 0.06)] = P
    return st, lp
