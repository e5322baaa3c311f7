"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) with the same method
names as multiraft_amd.engine.Engine. Test infrastructure only."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from multiraft_amd._abi import (AE_ARGS, AE_REPLY, AE_RESULT, IS_ARGS, IS_REPLY, IS_RESULT,
                                PERSISTENT, RV_ARGS, RV_REPLY, RV_RESULT, MraftSoa, ptr, soa_of)
from multiraft_amd.engine import copy_state

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PATH = os.path.join(ROOT, "oracle", "liboracle.so")


class OraEngine(ctypes.Structure):
    _fields_ = [("G", ctypes.c_int32), ("P", ctypes.c_int32), ("L", ctypes.c_int32),
                ("s", MraftSoa)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(_PATH)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        E = ctypes.POINTER(OraEngine)
        sigs = {
            "ora_count_enable": [E], "ora_count_disable": [], "ora_count_result": [vp],
            "ora_count_result_lines": [i32, vp],
            "ora_compute_terms_sorted": [E],
            "ora_gather_append_args": [E, vp, vp, i64, vp, vp],
            "ora_handle_append_entries": [E, vp, i64, vp, i64, vp, vp],
            "ora_process_append_replies": [E, vp, i64, vp, i64, vp, vp],
            "ora_replicate_tick": [E, vp, vp],
            "ora_replicate_tick_mt": [E, vp, vp, i32],
            "ora_start": [E, vp, vp, i64, vp, vp, vp, vp],
            "ora_collect_apply": [E, vp, vp, vp, vp],
            "ora_start_election": [E, vp, i64, vp, vp],
            "ora_handle_request_vote": [E, vp, i64, vp, vp],
            "ora_process_vote_replies": [E, vp, i64, vp, i64, vp, vp],
            "ora_export_group_status": [E, vp, vp, vp],
            "ora_election_rounds": [E, vp, i32, vp],
            "ora_election_rounds_mt": [E, vp, i32, vp, i32],
            "ora_snapshot": [E, vp, vp, i64, vp],
            "ora_gather_install_snapshot_args": [E, vp, vp, i64, vp, vp],
            "ora_handle_install_snapshot": [E, vp, i64, vp, vp, vp],
            "ora_process_install_snapshot_replies": [E, vp, i64, vp, i64, vp, vp],
            "ora_collect_persist": [E, vp],
            "ora_read_persistent": [E, vp, i64, vp, vp, i64],
            "ora_restore": [E, vp, i64, vp, i64, vp],
            "goshape_build": [i32, i32, i32, ctypes.POINTER(MraftSoa)],
            "goshape_store": [vp, ctypes.POINTER(MraftSoa)],
            "goshape_free": [vp],
            "goshape_tick": [vp, vp, i32],
            "goshape_reset": [vp, ctypes.POINTER(MraftSoa), i32],
        }
        for n, a in sigs.items():
            f = getattr(l, n)
            f.argtypes = a
            f.restype = None if n in ("ora_count_disable", "ora_count_result", "ora_count_result_lines", "goshape_store",
                                      "goshape_free", "goshape_reset", "ora_compute_terms_sorted") else ctypes.c_int
        l.goshape_build.restype = ctypes.c_void_p
        l.goshape_tick.restype = ctypes.c_int64
        _lib = l
    return _lib


class Oracle:
    """CPU restatement with the Engine's interface; operates on its own copy
    of the state."""

    def __init__(self, G: int, P: int, L: int, st: dict):
        self.G, self.P, self.L = G, P, L
        self.st = copy_state(st)
        self.st.setdefault("log_head", np.zeros(G * P, np.int32))  # fixtures made before the ring
        self.st.setdefault("has_snapshot", np.zeros(G * P, np.int32))
        self.st["terms_sorted"] = np.zeros(G * P, np.int32)
        self._e = OraEngine(G, P, L, soa_of(self.st))
        lib().ora_compute_terms_sorted(ctypes.byref(self._e))  # as mraft_load_state does

    def state(self) -> dict:
        return self.st

    def replicate_tick(self, leader_peer, nthreads: int = 1):
        lp = np.ascontiguousarray(leader_peer, dtype=np.int32)
        gf = np.zeros(self.G, dtype=np.int32)
        if nthreads > 1:
            lib().ora_replicate_tick_mt(ctypes.byref(self._e), ptr(lp), ptr(gf), nthreads)
        else:
            lib().ora_replicate_tick(ctypes.byref(self._e), ptr(lp), ptr(gf))
        return gf

    def replicate_tick_count(self, leader_peer, line_words=()):
        """Counts on a scratch copy (the state is left untouched). With
        line_words, also {line_words: (read lines, written lines)}."""
        scratch = Oracle(self.G, self.P, self.L, self.st)
        L = lib()
        L.ora_count_enable(ctypes.byref(scratch._e))
        lines = {}
        try:
            gf = scratch.replicate_tick(leader_peer)
            out = (ctypes.c_int64 * 2)()
            L.ora_count_result(out)
            for lw in line_words:
                o2 = (ctypes.c_int64 * 2)()
                L.ora_count_result_lines(lw, o2)
                lines[lw] = (int(o2[0]), int(o2[1]))
        finally:
            L.ora_count_disable()
        active = int(np.count_nonzero(gf & 1))
        if line_words:
            return int(out[0]), int(out[1]), active, lines
        return int(out[0]), int(out[1]), active

    def gather_append_args(self, slots, peers):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=AE_ARGS)
        err = np.zeros(n, dtype=np.int32)
        lib().ora_gather_append_args(ctypes.byref(self._e), ptr(slots), ptr(peers), n, ptr(out), ptr(err))
        return out, err

    def handle_append_entries(self, args, entry_terms):
        args = np.ascontiguousarray(args, dtype=AE_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=AE_REPLY)
        err = np.zeros(n, dtype=np.int32)
        et = None if entry_terms is None else np.ascontiguousarray(entry_terms, dtype=np.int32)
        lib().ora_handle_append_entries(ctypes.byref(self._e), ptr(args), n, ptr(et),
                                        0 if et is None else len(et), ptr(rep), ptr(err))
        return rep, err

    def process_append_replies(self, items, seg_begin=None):
        items = np.ascontiguousarray(items, dtype=AE_RESULT)
        n = len(items)
        flags = np.zeros(n, dtype=np.int32)
        err = np.zeros(n, dtype=np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        lib().ora_process_append_replies(ctypes.byref(self._e), ptr(items), n, ptr(sb),
                                         0 if sb is None else len(sb) - 1, ptr(flags), ptr(err))
        return flags, err

    def start(self, slots, counts=None):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        c = None if counts is None else np.ascontiguousarray(counts, dtype=np.int32)
        idx, term, isl, err = (np.zeros(n, np.int32) for _ in range(4))
        lib().ora_start(ctypes.byref(self._e), ptr(slots), ptr(c), n, ptr(idx), ptr(term), ptr(isl), ptr(err))
        return idx, term, isl, err

    def collect_apply(self, snapshots: bool = False):
        gp = self.G * self.P
        fr, to = np.zeros(gp, np.int32), np.zeros(gp, np.int32)
        si = np.zeros(gp, np.int32) if snapshots else None
        stm = np.zeros(gp, np.int32) if snapshots else None
        lib().ora_collect_apply(ctypes.byref(self._e), ptr(fr), ptr(to), ptr(si), ptr(stm))
        return (fr, to, si, stm) if snapshots else (fr, to)

    def store_state(self):
        return copy_state(self.st)

    def scalar_state(self):
        """The live state arrays (read-only use: the harness's mirror)."""
        return self.st

    # ---- snapshots ---------------------------------------------------------
    def snapshot(self, slots, index):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        index = np.ascontiguousarray(index, dtype=np.int32)
        err = np.zeros(len(slots), np.int32)
        lib().ora_snapshot(ctypes.byref(self._e), ptr(slots), ptr(index), len(slots), ptr(err))
        return err

    def gather_install_snapshot_args(self, slots, peers):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=IS_ARGS)
        err = np.zeros(n, np.int32)
        lib().ora_gather_install_snapshot_args(ctypes.byref(self._e), ptr(slots), ptr(peers), n, ptr(out), ptr(err))
        return out, err

    def handle_install_snapshot(self, args):
        args = np.ascontiguousarray(args, dtype=IS_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=IS_REPLY)
        fl = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        lib().ora_handle_install_snapshot(ctypes.byref(self._e), ptr(args), n, ptr(rep), ptr(fl), ptr(err))
        return rep, fl, err

    def process_install_snapshot_replies(self, items, seg_begin=None):
        items = np.ascontiguousarray(items, dtype=IS_RESULT)
        n = len(items)
        fl = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        lib().ora_process_install_snapshot_replies(ctypes.byref(self._e), ptr(items), n, ptr(sb),
                                                   0 if sb is None else len(sb) - 1, ptr(fl), ptr(err))
        return fl, err

    def start_election(self, slots):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=RV_ARGS)
        err = np.zeros(n, dtype=np.int32)
        lib().ora_start_election(ctypes.byref(self._e), ptr(slots), n, ptr(out), ptr(err))
        return out, err

    def handle_request_vote(self, args):
        args = np.ascontiguousarray(args, dtype=RV_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=RV_REPLY)
        err = np.zeros(n, dtype=np.int32)
        lib().ora_handle_request_vote(ctypes.byref(self._e), ptr(args), n, ptr(rep), ptr(err))
        return rep, err

    def process_vote_replies(self, items, seg_begin=None):
        items = np.ascontiguousarray(items, dtype=RV_RESULT)
        n = len(items)
        flags = np.zeros(n, dtype=np.int32)
        err = np.zeros(n, dtype=np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        lib().ora_process_vote_replies(ctypes.byref(self._e), ptr(items), n, ptr(sb),
                                       0 if sb is None else len(sb) - 1, ptr(flags), ptr(err))
        return flags, err

    def election_rounds(self, cand_mask, nthreads: int = 1):
        m = np.ascontiguousarray(cand_mask, dtype=np.uint8)
        gf = np.zeros(self.G, np.int32)
        lib().ora_election_rounds_mt(ctypes.byref(self._e), ptr(m), m.shape[0], ptr(gf), nthreads)
        return gf

    # ---- persistence ---------------------------------------------------------
    def collect_persist(self):
        out = np.zeros(self.G * self.P, np.int32)
        lib().ora_collect_persist(ctypes.byref(self._e), ptr(out))
        return out

    def read_persistent(self, slots):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        hdr = np.zeros(n, dtype=PERSISTENT)
        cap = max(1, n * self.L)
        terms = np.zeros(cap, np.int32)
        rc = lib().ora_read_persistent(ctypes.byref(self._e), ptr(slots), n, ptr(hdr), ptr(terms), cap)
        assert rc == 0
        used = int((hdr["last_index"] - hdr["dummy_index"] + 1).sum()) if n else 0
        return hdr, terms[:used].copy()

    def restore(self, hdr, terms):
        hdr = np.ascontiguousarray(hdr, dtype=PERSISTENT)
        terms = np.ascontiguousarray(terms, dtype=np.int32)
        err = np.zeros(len(hdr), np.int32)
        lib().ora_restore(ctypes.byref(self._e), ptr(hdr), len(hdr), ptr(terms), len(terms), ptr(err))
        return err

    def export_group_status(self, leader_peer=None):
        commit = np.zeros(self.G, dtype=np.int32)
        tl = np.zeros(self.G, dtype=np.int32)
        lp = None if leader_peer is None else np.ascontiguousarray(leader_peer, dtype=np.int32)
        lib().ora_export_group_status(ctypes.byref(self._e), ptr(lp), ptr(commit), ptr(tl))
        return commit, tl


def logical_logs(st: dict, G: int, P: int, L: int):
    """[G*P, L] view of every replica's log in Index order: row r, column k =
    the term of Index dummy + k (the ring of include/mraft.h unrolled from
    log_head); columns past last - dummy are dead slots."""
    lt = st["log_term"].reshape(G * P, L)
    h = st["log_head"] if "log_head" in st else np.zeros(G * P, np.int32)
    cols = (h[:, None].astype(np.int64) + np.arange(L)[None, :]) % L
    return np.take_along_axis(lt, cols, axis=1)


def assert_states_equal(a: dict, b: dict, G: int, P: int, L: int, ctx: str = "", heads: bool = True):
    """Compare two state images. Logs are compared in Index order over the
    live entries [dummy, last] of every replica (slots past lastIndex are dead:
    the reference's slice has no such slots). heads=False skips the ring
    positions themselves (the Python restatement has no ring)."""
    for st in (a, b):
        assert_terms_sorted_sound(st, G, P, L, ctx)
    for k in a:
        if k == "log_term" or (k == "log_head" and not heads) or k not in b:
            continue
        if not np.array_equal(a[k], b[k]):
            bad = np.nonzero(a[k] != b[k])[0][:8]
            raise AssertionError(f"{ctx}: {k} differs at {bad}: {a[k][bad]} vs {b[k][bad]}")
    la = logical_logs(a, G, P, L)
    lb = logical_logs(b, G, P, L)
    live = a["last_index"] - a["dummy_index"]
    mask = np.arange(L)[None, :] <= live[:, None]
    if not np.array_equal(np.where(mask, la, 0), np.where(mask, lb, 0)):
        rows = np.nonzero((np.where(mask, la, 0) != np.where(mask, lb, 0)).any(axis=1))[0][:8]
        raise AssertionError(f"{ctx}: log_term differs in replicas {rows}")


def terms_sorted_exact(st: dict, G: int, P: int, L: int) -> np.ndarray:
    """Whether each replica's terms of Index dummy+1 .. last never decrease."""
    logs = logical_logs(st, G, P, L).astype(np.int64)
    live = (st["last_index"] - st["dummy_index"]).astype(np.int64)  # entries after the dummy
    k = np.arange(1, L)[None, :]
    desc = (logs[:, 1:-1] > logs[:, 2:]) if L > 2 else np.zeros((G * P, 0), bool)
    desc = desc & (k[:, :-1] < live[:, None]) if L > 2 else desc
    return (~desc.any(axis=1)).astype(np.int32)


def assert_terms_sorted_sound(st: dict, G: int, P: int, L: int, ctx: str = ""):
    """terms_sorted is a proof (include/mraft.h): 1 only where the terms after
    the dummy really never decrease."""
    if "terms_sorted" not in st:
        return
    bad = np.nonzero((st["terms_sorted"] != 0) & (terms_sorted_exact(st, G, P, L) == 0))[0]
    if len(bad):
        raise AssertionError(f"{ctx}: terms_sorted claims sorted terms in replicas {bad[:8]}")


def rotate_rings(st: dict, G: int, P: int, L: int, rng, frac: float = 1.0) -> dict:
    """The same logical state with every replica's ring started at a random
    head (a fraction `frac` of the replicas): row contents rotated so Index
    dummy + k sits at (head + k) mod L. Exercises the wrap in every kernel."""
    out = {k: np.array(v, copy=True) for k, v in st.items()}
    logs = logical_logs(st, G, P, L)
    h = rng.integers(0, L, G * P).astype(np.int32)
    h[rng.random(G * P) >= frac] = 0
    cols = (h[:, None].astype(np.int64) + np.arange(L)[None, :]) % L
    lt = np.empty_like(logs)
    np.put_along_axis(lt, cols, logs, axis=1)
    out["log_term"] = lt.reshape(-1)
    out["log_head"] = h
    return out


class GoShaped:
    """The tick on the reference's own data shapes (oracle/mraft_goshape.c):
    the CPU baseline's Go-shaped variant. Built from a SoA image (untimed)."""

    def __init__(self, G: int, P: int, L: int, st: dict):
        self.G, self.P, self.L = G, P, L
        self._st = st
        self._soa = soa_of(st)
        self._c = lib().goshape_build(G, P, L, ctypes.byref(self._soa))

    def replicate_tick(self, leader_peer, nthreads: int = 1) -> int:
        lp = np.ascontiguousarray(leader_peer, dtype=np.int32)
        return int(lib().goshape_tick(self._c, ptr(lp), nthreads))

    def reset(self, nthreads: int = 1):
        """Back to the state it was built from (slices keep their capacity)."""
        lib().goshape_reset(self._c, ctypes.byref(self._soa), nthreads)

    def state(self) -> dict:
        out = copy_state(self._st)
        soa = soa_of(out)
        lib().goshape_store(self._c, ctypes.byref(soa))
        return out

    def close(self):
        if self._c:
            lib().goshape_free(self._c)
            self._c = None

    def __del__(self):
        self.close()


def random_reply_segments(st: dict, G: int, P: int, lp: np.ndarray, seed: int, max_len: int = 150):
    """Reply batches for process_append_replies beyond what a3 produces: per
    leader slot a segment of 0..max_len replies in arrival order (repeats of a
    peer, stale and higher terms, failures, successes whose matchIndex moves
    up and down), so a1 runs many times per segment, over logs whose tail may
    not carry the current term (the Figure-8 scan). Returns items, seg_begin."""
    rng = np.random.default_rng(seed)
    L = st["log_term"].size // (G * P)
    out = []
    seg = [0]
    for g in range(G):
        if lp[g] < 0 or P < 2:
            continue
        s = g * P + int(lp[g])
        k = int(rng.integers(0, max_len + 1)) if rng.random() < 0.9 else 0
        T, last = int(st["current_term"][s]), int(st["last_index"][s])
        nxt = st["next_index"][s * P:(s + 1) * P].astype(np.int64).copy()
        for _ in range(k):
            p = int(rng.integers(0, P - 1))
            p = p if p < s % P else p + 1
            r = np.zeros(1, dtype=AE_RESULT)[0]
            r["slot"], r["peer"] = s, p
            u = rng.random()
            r["args_term"] = T if u < 0.9 else T - 1
            prev = int(nxt[p]) - 1 if rng.random() < 0.8 else int(rng.integers(0, last + 1))
            r["args_prev_log_index"] = prev
            n = int(rng.integers(0, max(1, last - prev + 1))) if prev <= last else 0
            r["args_n_entries"] = n
            v = rng.random()
            r["reply_term"] = T if v < 0.995 else (T + 1 if v < 0.997 else T - 1)
            ok = rng.random() < 0.7
            r["reply_success"] = int(ok)
            r["reply_conflict_index"] = int(rng.integers(1, max(2, prev + 2)))
            if ok and prev == nxt[p] - 1:
                nxt[p] = prev + n + 1
            elif prev == nxt[p] - 1:
                nxt[p] = r["reply_conflict_index"]
            out.append(r)
        seg.append(len(out))
    items = np.array(out, dtype=AE_RESULT) if out else np.zeros(0, dtype=AE_RESULT)
    return items, np.array(seg, dtype=np.int64)
