"""Host-side mirror of the engine boundary (include/mraft.h) over ctypes.

`Engine` wraps one libmraft_hip.so handle: G groups x P peers of Raft replica
state resident in HBM, and the batched decision entry points that replace the
reference's per-instance handlers (src/raft/raft_append_entry.go,
src/raft/raft_election.go). Host batches are numpy arrays of the structured
dtypes in `_abi` (synchronous calls); device batches are torch tensors or raw
device addresses (asynchronous on the engine's stream).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _abi
from ._abi import (AE_ARGS, AE_REPLY, AE_RESULT, IS_ARGS, IS_REPLY, IS_RESULT, PERSISTENT, RV_ARGS,
                   RV_REPLY, RV_RESULT, DEVICE, HOST, STATE_FIELDS, ptr, soa_of)


class MraftError(RuntimeError):
    pass


def _ck(rc: int, what: str):
    if rc != _abi.OK:
        raise MraftError(f"{what} failed ({rc}): {_abi.last_error()}")


def state_sizes(G: int, P: int, L: int) -> dict:
    gp = G * P
    return {f: (gp * L if f == "log_term" else gp * P if f in ("match_index", "next_index") else gp)
            for f in STATE_FIELDS}


def new_state(G: int, P: int, L: int) -> dict:
    """A host state image initialised as Make does (raft.go:51-87)."""
    st = {f: np.zeros(n, dtype=np.int32) for f, n in state_sizes(G, P, L).items()}
    st["voted_for"][:] = -1
    st["state"][:] = _abi.FOLLOWER
    st["terms_sorted"][:] = 1  # [dummy] only
    return st


def copy_state(st: dict) -> dict:
    return {k: np.array(v, copy=True) for k, v in st.items()}


def entry_positions(log_head, L: int, entries_offset, n_entries) -> np.ndarray:
    """Where, in a host copy of `log_term` ([G*P*L], include/mraft.h), the
    entries an AppendEntries names by reference are: mraft_gather_append_args
    sets entries_offset = slot * L + (prev + 1 - dummyIndex), the LOGICAL
    position in that replica's ring, so entry k of item i is at
    slot * L + (log_head[slot] + pos + k) mod L. Returns the flat indices of
    every item's entries, item after item (a host shipping entries over the
    network copies log_term[entry_positions(...)])."""
    eo = np.asarray(entries_offset, dtype=np.int64)
    n = np.maximum(np.asarray(n_entries, dtype=np.int64), 0)
    slot, pos = eo // L, eo % L
    item = np.repeat(np.arange(len(eo)), n)
    within = np.arange(int(n.sum()), dtype=np.int64) - np.repeat(np.cumsum(n) - n, n)
    head = np.asarray(log_head, dtype=np.int64)[slot][item]
    return slot[item] * L + (head + pos[item] + within) % L


def synth_tick_state(G: int, P: int, L: int, seed: int, g_begin: int = 0, g_end: int | None = None,
                     nthreads: int | None = None):
    """Seeded replication-tick workload (include/mraft_synth.h). Returns
    (state, leader_peer, item_class) for groups [g_begin, g_end)."""
    g_end = G if g_end is None else g_end
    n = g_end - g_begin
    st = {f: np.empty(sz, dtype=np.int32) for f, sz in state_sizes(n, P, L).items()}
    lp = np.empty(n, dtype=np.int32)
    ic = np.empty(n * P, dtype=np.int32)
    soa = soa_of(st)
    nt = nthreads if nthreads is not None else min(16, os.cpu_count() or 1)
    rc = _abi.synth().mraft_synth_tick_state(seed, G, P, L, g_begin, g_end, ctypes.byref(soa),
                                             ptr(lp), ptr(ic), nt)
    if rc != 0:
        raise MraftError(f"mraft_synth_tick_state failed ({rc})")
    return st, lp, ic


def synth_election_state(G: int, P: int, L: int, seed: int, rounds: int, g_begin: int = 0,
                         g_end: int | None = None, nthreads: int | None = None):
    """Seeded election-storm workload (config #5): (state, cand_mask[rounds, n])."""
    g_end = G if g_end is None else g_end
    n = g_end - g_begin
    st = {f: np.empty(sz, dtype=np.int32) for f, sz in state_sizes(n, P, L).items()}
    mask = np.zeros((rounds, n), dtype=np.uint8)
    soa = soa_of(st)
    nt = nthreads if nthreads is not None else min(16, os.cpu_count() or 1)
    rc = _abi.synth().mraft_synth_election_state(seed, G, P, L, g_begin, g_end, ctypes.byref(soa),
                                                 ptr(mask), rounds, nt)
    if rc != 0:
        raise MraftError(f"mraft_synth_election_state failed ({rc})")
    return st, mask


def synth_fold_batch(st: dict, G: int, P: int, L: int, leader_peer: np.ndarray, seed: int):
    items = np.zeros(G * max(P - 1, 0), dtype=AE_RESULT)
    seg = np.zeros(G + 1, dtype=np.int64)
    soa = soa_of(st)
    n = _abi.synth().mraft_synth_fold_batch(seed, G, P, L, ctypes.byref(soa), ptr(leader_peer),
                                            ptr(items), ptr(seg))
    return items[:n], seg


class Engine:
    """One engine handle per GPU (calls must be serialized by the caller)."""

    def __init__(self, G: int, P: int, L: int, device: int = 0, alloc: bool = True,
                 dedicated_queue: bool = False):
        self.G, self.P, self.L = G, P, L
        self._lib = _abi.lib()
        h = ctypes.c_void_p()
        flags = (0 if alloc else _abi.CREATE_NO_ALLOC) | (_abi.CREATE_DEDICATED_QUEUE if dedicated_queue else 0)
        _ck(self._lib.mraft_create(G, P, L, device, flags, ctypes.byref(h)), "mraft_create")
        self._h = h

    # ---- lifetime --------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.mraft_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int | None):
        _ck(self._lib.mraft_set_stream(self._h, stream_ptr), "mraft_set_stream")

    def stream(self) -> int:
        return self._lib.mraft_get_stream(self._h) or 0

    def synchronize(self):
        _ck(self._lib.mraft_synchronize(self._h), "mraft_synchronize")

    def set_tick_shards(self, shards: int):
        """Tick group shards on engine-owned hardware queues (mraft_set_tick_shards)."""
        _ck(self._lib.mraft_set_tick_shards(self._h, shards), "mraft_set_tick_shards")

    def tick_shards(self) -> int:
        return int(self._lib.mraft_get_tick_shards(self._h))

    def set_tick_mode(self, mode: int):
        """TICK_FULL, TICK_LIGHT or TICK_AUTO (the default; mraft_set_tick_mode):
        the light tick settles steady-state groups eight per wave and runs the
        rest through the full tick; AUTO picks per shard from the last light
        tick's fallback share. Outputs are identical in every mode."""
        _ck(self._lib.mraft_set_tick_mode(self._h, mode), "mraft_set_tick_mode")

    def tick_mode(self) -> int:
        return int(self._lib.mraft_get_tick_mode(self._h))

    def tick_light_fallbacks(self) -> int:
        """Groups the last completed light tick sent to the full tick (-1: none yet)."""
        return int(self._lib.mraft_tick_light_fallbacks(self._h))

    def set_stage_capacity(self, words: int):
        """Words of staged entries mraft_handle_append_entries may use for its
        deferred items (mraft_set_stage_capacity; 0 forces the ordered fallback)."""
        _ck(self._lib.mraft_set_stage_capacity(self._h, words), "mraft_set_stage_capacity")

    def stage_capacity(self) -> int:
        return int(self._lib.mraft_get_stage_capacity(self._h))

    def shard_stream(self, shard: int) -> int:
        return self._lib.mraft_shard_stream(self._h, shard) or 0

    # ---- state -----------------------------------------------------------
    def load_state(self, st: dict, where: int = HOST):
        if where == HOST:  # images made before the ring / hasSnapshot / terms_sorted (recomputed on load)
            for f in ("log_head", "has_snapshot", "terms_sorted"):
                if f not in st:
                    st = dict(st, **{f: np.zeros(self.G * self.P, np.int32)})
        soa = soa_of(st)
        _ck(self._lib.mraft_load_state(self._h, ctypes.byref(soa), where), "mraft_load_state")

    def store_state(self) -> dict:
        out = {f: np.empty(n, dtype=np.int32) for f, n in state_sizes(self.G, self.P, self.L).items()}
        soa = soa_of(out)
        _ck(self._lib.mraft_store_state(self._h, ctypes.byref(soa), HOST), "mraft_store_state")
        return out

    def scalar_state(self, fields=("current_term", "voted_for", "state", "commit_index", "last_applied",
                                   "dummy_index", "last_index", "log_head", "has_snapshot")) -> dict:
        """The per-replica scalar arrays only (no logs, no leader view): a
        cheap host mirror of roles and terms (mraft_store_state with the
        other arrays NULL)."""
        out = {f: np.empty(self.G * self.P, dtype=np.int32) for f in fields}
        soa = soa_of(out)
        _ck(self._lib.mraft_store_state(self._h, ctypes.byref(soa), HOST), "mraft_store_state")
        return out

    def view(self) -> dict:
        soa = _abi.MraftSoa()
        _ck(self._lib.mraft_state_view(self._h, ctypes.byref(soa)), "mraft_state_view")
        return {f: getattr(soa, f) for f in STATE_FIELDS}

    def bind(self, dev_state: dict):
        soa = soa_of(dev_state)
        _ck(self._lib.mraft_bind_state(self._h, ctypes.byref(soa)), "mraft_bind_state")

    # ---- hot path --------------------------------------------------------
    def replicate_tick(self, leader_peer, group_flags=None, where: int = HOST):
        if where == HOST:
            leader_peer = np.ascontiguousarray(leader_peer, dtype=np.int32)
            if group_flags is None:
                group_flags = np.zeros(self.G, dtype=np.int32)
        _ck(self._lib.mraft_replicate_tick(self._h, ptr(leader_peer), ptr(group_flags), where),
            "mraft_replicate_tick")
        return group_flags

    def start_and_tick(self, leader_peer, counts, group_flags=None, where: int = HOST):
        """Start (raft.go:90-104) of counts[g] entries at every group's leader
        replica, then the tick (mraft_start_and_tick). Host arrays: returns
        (group_flags, (index, term, is_leader, err)), Start's outputs per group."""
        G = self.G
        if where == HOST:
            leader_peer = np.ascontiguousarray(leader_peer, dtype=np.int32)
            counts = np.ascontiguousarray(counts, dtype=np.int32)
            if group_flags is None:
                group_flags = np.zeros(G, dtype=np.int32)
            outs = tuple(np.zeros(G, np.int32) for _ in range(4))
        else:
            import torch
            outs = tuple(torch.empty(G, dtype=torch.int32, device=leader_peer.device) for _ in range(4))
        _ck(self._lib.mraft_start_and_tick(self._h, ptr(leader_peer), ptr(counts), ptr(outs[0]), ptr(outs[1]),
                                           ptr(outs[2]), ptr(outs[3]), ptr(group_flags), where),
            "mraft_start_and_tick")
        return group_flags, outs

    def replicate_tick_export(self, leader_peer, group_flags=None, commit=None, term_leader=None,
                              where: int = HOST):
        """The tick with the GetState export fused in: (flags, commit, term<<1|leader)."""
        if where == HOST:
            leader_peer = np.ascontiguousarray(leader_peer, dtype=np.int32)
            if group_flags is None:
                group_flags = np.zeros(self.G, dtype=np.int32)
            if commit is None:
                commit = np.zeros(self.G, dtype=np.int32)
            if term_leader is None:
                term_leader = np.zeros(self.G, dtype=np.int32)
        _ck(self._lib.mraft_replicate_tick_export(self._h, ptr(leader_peer), ptr(group_flags),
                                                  ptr(commit), ptr(term_leader), where),
            "mraft_replicate_tick_export")
        return group_flags, commit, term_leader

    def replicate_tick_count(self, leader_peer, where: int = HOST):
        if where == HOST:
            leader_peer = np.ascontiguousarray(leader_peer, dtype=np.int32)
        out = (ctypes.c_int64 * 3)()
        _ck(self._lib.mraft_replicate_tick_count(self._h, ptr(leader_peer), out, where),
            "mraft_replicate_tick_count")
        return int(out[0]), int(out[1]), int(out[2])

    def gather_append_args(self, slots, peers):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=AE_ARGS)
        err = np.zeros(n, dtype=np.int32)
        _ck(self._lib.mraft_gather_append_args(self._h, ptr(slots), ptr(peers), n, ptr(out),
                                               ptr(err), HOST), "mraft_gather_append_args")
        return out, err

    def handle_append_entries(self, args: np.ndarray, entry_terms: np.ndarray | None, results: bool = False):
        """HandleAppendEntries for a batch: (replies, item_err), and with
        results=True also the reply records the co-resident leaders fold
        (mraft_handle_append_entries_ex)."""
        args = np.ascontiguousarray(args, dtype=AE_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=AE_REPLY)
        err = np.zeros(n, dtype=np.int32)
        res = np.zeros(n, dtype=AE_RESULT) if results else None
        et = None if entry_terms is None else np.ascontiguousarray(entry_terms, dtype=np.int32)
        _ck(self._lib.mraft_handle_append_entries_ex(self._h, ptr(args), n, ptr(et),
                                                     0 if et is None else len(et), ptr(rep), ptr(res),
                                                     ptr(err), HOST), "mraft_handle_append_entries_ex")
        return (rep, err, res) if results else (rep, err)

    def process_append_replies(self, items: np.ndarray, seg_begin: np.ndarray | None = None):
        items = np.ascontiguousarray(items, dtype=AE_RESULT)
        n = len(items)
        flags = np.zeros(n, dtype=np.int32)
        err = np.zeros(n, dtype=np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        _ck(self._lib.mraft_process_append_replies(self._h, ptr(items), n, ptr(sb),
                                                   0 if sb is None else len(sb) - 1, ptr(flags),
                                                   ptr(err), HOST),
            "mraft_process_append_replies")
        return flags, err

    def start(self, slots, counts=None):
        """Start (raft.go:90-104): returns (index, term, is_leader, err)."""
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        c = None if counts is None else np.ascontiguousarray(counts, dtype=np.int32)
        idx = np.zeros(n, np.int32)
        term = np.zeros(n, np.int32)
        isl = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        _ck(self._lib.mraft_start(self._h, ptr(slots), ptr(c), n, ptr(idx), ptr(term), ptr(isl),
                                  ptr(err), HOST), "mraft_start")
        return idx, term, isl, err

    def collect_apply(self, snapshots: bool = False):
        """Applier (raft.go:153-203): per-slot ApplyMsg index ranges [from, to];
        with snapshots=True also (snap_index, snap_term): the SnapshotValid
        message each slot sends first (snap_index -1: none)."""
        gp = self.G * self.P
        fr = np.zeros(gp, np.int32)
        to = np.zeros(gp, np.int32)
        si = np.zeros(gp, np.int32) if snapshots else None
        stm = np.zeros(gp, np.int32) if snapshots else None
        _ck(self._lib.mraft_collect_apply(self._h, ptr(fr), ptr(to), ptr(si), ptr(stm), HOST),
            "mraft_collect_apply")
        return (fr, to, si, stm) if snapshots else (fr, to)

    def collect_apply_compact(self, cap: int | None = None, snapshots: bool = False):
        """Applier, compacted: (slots, from, to, total) for the slots with a
        message to send (hasSnapshot or commitIndex > lastApplied), ascending;
        only the returned ones advance. snapshots=True returns (slots,
        snap_index, snap_term, from, to, total)."""
        cap = self.G * self.P if cap is None else cap
        sl, si, stm, fr, to = (np.zeros(max(cap, 1), np.int32) for _ in range(5))
        n = np.zeros(1, np.int64)
        # without snapshots the SnapshotValid outputs are NULL: hasSnapshot
        # stays set (and snapshot-only slots do not count) until a call that
        # takes them, as in collect_apply(snapshots=False)
        _ck(self._lib.mraft_collect_apply_compact(self._h, ptr(sl), ptr(si) if snapshots else None,
                                                  ptr(stm) if snapshots else None, ptr(fr), ptr(to), cap,
                                                  ptr(n), HOST), "mraft_collect_apply_compact")
        k = int(min(n[0], cap))
        if snapshots:
            return sl[:k].copy(), si[:k].copy(), stm[:k].copy(), fr[:k].copy(), to[:k].copy(), int(n[0])
        return sl[:k].copy(), fr[:k].copy(), to[:k].copy(), int(n[0])

    # ---- snapshots (raft_snapshot.go) -------------------------------------
    def snapshot(self, slots, index):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        index = np.ascontiguousarray(index, dtype=np.int32)
        err = np.zeros(len(slots), np.int32)
        _ck(self._lib.mraft_snapshot(self._h, ptr(slots), ptr(index), len(slots), ptr(err), HOST),
            "mraft_snapshot")
        return err

    def gather_install_snapshot_args(self, slots, peers):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=IS_ARGS)
        err = np.zeros(n, np.int32)
        _ck(self._lib.mraft_gather_install_snapshot_args(self._h, ptr(slots), ptr(peers), n, ptr(out),
                                                         ptr(err), HOST),
            "mraft_gather_install_snapshot_args")
        return out, err

    def handle_install_snapshot(self, args):
        args = np.ascontiguousarray(args, dtype=IS_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=IS_REPLY)
        fl = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        _ck(self._lib.mraft_handle_install_snapshot(self._h, ptr(args), n, ptr(rep), ptr(fl), ptr(err),
                                                    HOST), "mraft_handle_install_snapshot")
        return rep, fl, err

    def process_install_snapshot_replies(self, items, seg_begin=None):
        items = np.ascontiguousarray(items, dtype=IS_RESULT)
        n = len(items)
        fl = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        _ck(self._lib.mraft_process_install_snapshot_replies(
            self._h, ptr(items), n, ptr(sb), 0 if sb is None else len(sb) - 1, ptr(fl), ptr(err), HOST),
            "mraft_process_install_snapshot_replies")
        return fl, err

    # ---- elections -------------------------------------------------------
    def start_election(self, slots):
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        out = np.zeros(n, dtype=RV_ARGS)
        err = np.zeros(n, dtype=np.int32)
        _ck(self._lib.mraft_start_election(self._h, ptr(slots), n, ptr(out), ptr(err), HOST),
            "mraft_start_election")
        return out, err

    def handle_request_vote(self, args: np.ndarray):
        args = np.ascontiguousarray(args, dtype=RV_ARGS)
        n = len(args)
        rep = np.zeros(n, dtype=RV_REPLY)
        err = np.zeros(n, dtype=np.int32)
        _ck(self._lib.mraft_handle_request_vote(self._h, ptr(args), n, ptr(rep), ptr(err), HOST),
            "mraft_handle_request_vote")
        return rep, err

    def process_vote_replies(self, items: np.ndarray, seg_begin: np.ndarray | None = None):
        items = np.ascontiguousarray(items, dtype=RV_RESULT)
        n = len(items)
        flags = np.zeros(n, dtype=np.int32)
        err = np.zeros(n, dtype=np.int32)
        sb = None if seg_begin is None else np.ascontiguousarray(seg_begin, dtype=np.int64)
        _ck(self._lib.mraft_process_vote_replies(self._h, ptr(items), n, ptr(sb),
                                                 0 if sb is None else len(sb) - 1, ptr(flags),
                                                 ptr(err), HOST), "mraft_process_vote_replies")
        return flags, err

    def election_rounds(self, cand_mask, group_flags=None, where: int = HOST):
        """Election storm (config #5): len(cand_mask) rounds in one launch."""
        if where == HOST:
            cand_mask = np.ascontiguousarray(cand_mask, dtype=np.uint8)
            if group_flags is None:
                group_flags = np.zeros(self.G, dtype=np.int32)
            rounds = cand_mask.shape[0]
        else:
            rounds = cand_mask.shape[0]
        _ck(self._lib.mraft_election_rounds(self._h, ptr(cand_mask), rounds, ptr(group_flags), where),
            "mraft_election_rounds")
        return group_flags

    # ---- persistence (raft.go:205-235) ------------------------------------
    def collect_persist(self):
        """persist_dirty of every slot (MRAFT_PERSIST_* bits), cleared on read."""
        out = np.zeros(self.G * self.P, np.int32)
        _ck(self._lib.mraft_collect_persist(self._h, ptr(out), HOST), "mraft_collect_persist")
        return out

    def read_persistent(self, slots):
        """SaveState (raft.go:209-216) of the given slots: (PERSISTENT records,
        packed log terms)."""
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        n = len(slots)
        hdr = np.zeros(n, dtype=PERSISTENT)
        if n == 0:
            return hdr, np.zeros(0, np.int32)
        cap = n * self.L
        terms = np.zeros(cap, np.int32)
        _ck(self._lib.mraft_read_persistent(self._h, ptr(slots), n, ptr(hdr), ptr(terms), cap),
            "mraft_read_persistent")
        used = int(hdr["terms_offset"][-1] + hdr["last_index"][-1] - hdr["dummy_index"][-1] + 1)
        return hdr, terms[:used].copy()

    def restore(self, hdr, terms):
        """Crash + restart (Make + readPersist, raft.go:51-87,217-235)."""
        hdr = np.ascontiguousarray(hdr, dtype=PERSISTENT)
        terms = np.ascontiguousarray(terms, dtype=np.int32)
        err = np.zeros(len(hdr), np.int32)
        _ck(self._lib.mraft_restore(self._h, ptr(hdr), len(hdr), ptr(terms), len(terms), ptr(err)),
            "mraft_restore")
        return err

    def export_group_status(self, leader_peer=None):
        commit = np.zeros(self.G, dtype=np.int32)
        tl = np.zeros(self.G, dtype=np.int32)
        lp = None if leader_peer is None else np.ascontiguousarray(leader_peer, dtype=np.int32)
        _ck(self._lib.mraft_export_group_status(self._h, ptr(lp), ptr(commit), ptr(tl), HOST),
            "mraft_export_group_status")
        return commit, tl


    # ---- multi-GPU fan-in (include/mraft.h) -----------------
    def comm_init(self, nranks: int, rank: int, uid: bytes) -> int:
        """ncclCommInitRank on this engine's device (collective over the ranks):
        returns the ncclComm_t as an integer handle."""
        if len(uid) != _abi.COMM_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        c = ctypes.c_void_p()
        _ck(self._lib.mraft_comm_init(self._h, nranks, rank, ctypes.addressof(buf), ctypes.byref(c)),
            "mraft_comm_init")
        return c.value

    def allgather_status(self, comm: int, local, gathered=None, where: int = DEVICE,
                         overlap: bool = False, ordered: bool = False):
        """All-gather this rank's [2*G] status block (commit | term<<1|leader)
        into the [nranks*2*G] rank-major `gathered` buffer over RCCL.
        ordered: the caller has already made the fan-in stream wait for the
        producer of `local` (MRAFT_FANIN_ORDERED: no event recorded here)."""
        if where == HOST:
            local = np.ascontiguousarray(local, dtype=np.int32)
        _ck(self._lib.mraft_allgather_status(self._h, comm, ptr(local), ptr(gathered), where,
                                             _abi.FANIN_ORDERED if ordered else
                                             (_abi.FANIN_OVERLAP if overlap else 0)),
            "mraft_allgather_status")
        return gathered

    def fanin_synchronize(self):
        _ck(self._lib.mraft_fanin_synchronize(self._h), "mraft_fanin_synchronize")

    def fanin_stream(self) -> int:
        return self._lib.mraft_fanin_stream(self._h) or 0

    def fanin_reserve_cus(self, n_cus: int):
        _ck(self._lib.mraft_fanin_reserve_cus(self._h, n_cus), "mraft_fanin_reserve_cus")


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (mraft_comm_unique_id): 128 bootstrap bytes one rank
    creates and the host ships to the others over its own control plane."""
    buf = ctypes.create_string_buffer(_abi.COMM_ID_BYTES)
    _ck(_abi.lib().mraft_comm_unique_id(ctypes.addressof(buf)), "mraft_comm_unique_id")
    return buf.raw


def comm_destroy(comm: int):
    _ck(_abi.lib().mraft_comm_destroy(comm), "mraft_comm_destroy")


def export_group_status_into(eng: Engine, leader_peer, commit, term_leader, where: int = DEVICE):
    """GetState for every group into caller buffers (device tensors by default)."""
    _ck(eng._lib.mraft_export_group_status(eng._h, ptr(leader_peer), ptr(commit), ptr(term_leader),
                                           where), "mraft_export_group_status")


def encode_persistent(rec, terms) -> bytes:
    """One replica's persistent state as bytes (mraft_encode_persistent)."""
    r = np.zeros(1, dtype=PERSISTENT)
    for f in ("current_term", "voted_for", "dummy_index", "last_index"):
        r[f][0] = rec[f]
    r["terms_offset"][0] = 0
    t = np.ascontiguousarray(terms, dtype=np.int32)
    L = _abi.lib()
    size = L.mraft_encode_persistent(ptr(r), ptr(t), None, 0)
    if size < 0:
        raise MraftError(f"mraft_encode_persistent failed ({size})")
    buf = ctypes.create_string_buffer(size)
    got = L.mraft_encode_persistent(ptr(r), ptr(t), ctypes.addressof(buf), size)
    assert got == size
    return buf.raw


def decode_persistent(data: bytes):
    """Inverse of encode_persistent: (PERSISTENT record with slot 0, terms)."""
    r = np.zeros(1, dtype=PERSISTENT)
    cap = max(1, (len(data) - 36) // 8)
    terms = np.zeros(cap, np.int32)
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    rc = _abi.lib().mraft_decode_persistent(ctypes.addressof(buf), len(data), ptr(r), ptr(terms), cap)
    if rc != _abi.OK:
        raise MraftError(f"mraft_decode_persistent: malformed buffer ({rc})")
    n = int(r["last_index"][0] - r["dummy_index"][0] + 1)
    return r[0], terms[:n].copy()
