"""ctypes mirror of include/mraft.h and include/mraft_synth.h.

Loads the in-tree libmraft_hip.so (built by `make -C multiraft_amd/csrc` or
`__graft_entry__.build()`). There is no fallback: if the library is missing or
does not export the ABI, importing the engine raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRAFT_LIB") or os.path.join(_HERE, "libmraft_hip.so")
SYNTH_PATH = os.path.join(_HERE, "libmraft_synth.so")

# ---- constants (include/mraft.h) -------------------------------------------
LEADER, CANDIDATE, FOLLOWER = 1, 2, 3
HOST, DEVICE = 0, 1
TICK_FULL, TICK_LIGHT, TICK_AUTO = 0, 1, 2  # mraft_set_tick_mode
CREATE_NO_ALLOC = 1
CREATE_DEDICATED_QUEUE = 2
OK, E_INVAL, E_NOMEM, E_HIP, E_NOSTATE = 0, -1, -2, -3, -4
(ITEM_OK, ITEM_PREV_BEYOND_LAST, ITEM_BELOW_DUMMY, ITEM_LOG_FULL, ITEM_NEED_SNAPSHOT,
 ITEM_DUP_SLOT, ITEM_BAD_SLOT, ITEM_BAD_STATE) = range(8)
F_NEED_MORE, F_COMMITTED, F_STEPPED_DOWN, F_BECAME_LEADER, F_APPLIED = 1, 2, 4, 8, 16
F_SNAPSHOT_INSTALLED = 32
G_SNAPSHOT_INSTALLED = 256
(G_ACTIVE, G_COMMITTED, G_STEPPED_DOWN, G_NEED_SNAPSHOT, G_ERROR, G_FOLLOWER_COMMIT,
 G_LOG_FULL, G_ELECTED) = 1, 2, 4, 8, 16, 32, 64, 128
PERSIST_STATE, PERSIST_SNAPSHOT = 1, 2
TERMS_SORTED = 1
AE_ENTRIES_SORTED = 1
ABI_VERSION = 6
FANIN_OVERLAP = 1
FANIN_ORDERED = 2
COMM_ID_BYTES = 128
SYN_MATCH, SYN_MISMATCH, SYN_BEYOND, SYN_STALE, SYN_BELOW_DUMMY, SYN_HEARTBEAT = range(6)


def synth_seed(config_id: int) -> int:
    return 0xC0FFEE + config_id


# ---- structs ---------------------------------------------------------------
_P32 = ctypes.POINTER(ctypes.c_int32)

STATE_FIELDS = ("current_term", "voted_for", "state", "commit_index", "last_applied",
                "dummy_index", "last_index", "granted_votes", "log_term", "match_index",
                "next_index", "persist_dirty", "log_head", "has_snapshot", "terms_sorted")


class MraftSoa(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in STATE_FIELDS]


AE_ARGS = np.dtype([("slot", "<i4"), ("term", "<i4"), ("leader_id", "<i4"),
                    ("prev_log_index", "<i4"), ("prev_log_term", "<i4"),
                    ("leader_commit", "<i4"), ("n_entries", "<i4"), ("flags", "<i4"),
                    ("entries_offset", "<i8")])
AE_REPLY = np.dtype([("term", "<i4"), ("success", "<i4"), ("conflict_index", "<i4"),
                     ("conflict", "<i4")])
AE_RESULT = np.dtype([("slot", "<i4"), ("peer", "<i4"), ("args_term", "<i4"),
                      ("args_prev_log_index", "<i4"), ("args_n_entries", "<i4"),
                      ("reply_term", "<i4"), ("reply_success", "<i4"),
                      ("reply_conflict_index", "<i4")])
RV_ARGS = np.dtype([("slot", "<i4"), ("candidate_id", "<i4"), ("term", "<i4"),
                    ("last_log_index", "<i4"), ("last_log_term", "<i4")])
RV_REPLY = np.dtype([("term", "<i4"), ("vote_granted", "<i4")])
IS_ARGS = np.dtype([("slot", "<i4"), ("term", "<i4"), ("leader_id", "<i4"),
                    ("last_included_index", "<i4"), ("last_included_term", "<i4")])
IS_REPLY = np.dtype([("term", "<i4"), ("success", "<i4")])
IS_RESULT = np.dtype([("slot", "<i4"), ("peer", "<i4"), ("args_term", "<i4"),
                      ("args_last_included_index", "<i4"), ("reply_term", "<i4")])
RV_RESULT = np.dtype([("slot", "<i4"), ("peer", "<i4"), ("args_term", "<i4"),
                      ("reply_term", "<i4"), ("vote_granted", "<i4")])
PERSISTENT = np.dtype([("slot", "<i4"), ("current_term", "<i4"), ("voted_for", "<i4"),
                       ("dummy_index", "<i4"), ("last_index", "<i4"), ("_pad", "<i4"),
                       ("terms_offset", "<i8")])
assert PERSISTENT.itemsize == 32
assert AE_ARGS.itemsize == 40 and AE_RESULT.itemsize == 32 and RV_ARGS.itemsize == 20

# Every symbol include/mraft.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "mraft_create", "mraft_destroy", "mraft_set_stream", "mraft_get_stream",
    "mraft_synchronize", "mraft_dims", "mraft_last_error_string", "mraft_abi_version",
    "mraft_load_state", "mraft_store_state", "mraft_state_view", "mraft_bind_state",
    "mraft_gather_append_args", "mraft_handle_append_entries",
    "mraft_process_append_replies", "mraft_replicate_tick", "mraft_replicate_tick_count",
    "mraft_start", "mraft_collect_apply", "mraft_election_rounds",
    "mraft_snapshot", "mraft_gather_install_snapshot_args", "mraft_handle_install_snapshot",
    "mraft_process_install_snapshot_replies",
    "mraft_start_election", "mraft_handle_request_vote", "mraft_process_vote_replies",
    "mraft_export_group_status", "mraft_collect_persist", "mraft_read_persistent",
    "mraft_restore", "mraft_encode_persistent", "mraft_decode_persistent",
    "mraft_key2shard", "mraft_realloc_gid", "mraft_replicate_tick_export",
    "mraft_collect_apply_compact",
    "mraft_comm_unique_id", "mraft_comm_init", "mraft_comm_destroy", "mraft_allgather_status",
    "mraft_fanin_synchronize", "mraft_fanin_stream", "mraft_fanin_reserve_cus",
    "mraft_set_tick_shards", "mraft_get_tick_shards", "mraft_shard_stream", "mraft_handle_append_entries_ex",
    "mraft_set_stage_capacity", "mraft_get_stage_capacity",
    "mraft_set_tick_mode", "mraft_get_tick_mode", "mraft_tick_light_fallbacks", "mraft_start_and_tick",
)
SYNTH_SYMBOLS = ("mraft_synth_tick_state", "mraft_synth_fold_batch", "mraft_synth_election_state")

_vp, _i32, _i64, _u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
_SIGS = {
    "mraft_create": (ctypes.c_int, [_i32, _i32, _i32, _i32, _u32, ctypes.POINTER(_vp)]),
    "mraft_destroy": (ctypes.c_int, [_vp]),
    "mraft_set_stream": (ctypes.c_int, [_vp, _vp]),
    "mraft_get_stream": (_vp, [_vp]),
    "mraft_synchronize": (ctypes.c_int, [_vp]),
    "mraft_dims": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "mraft_last_error_string": (ctypes.c_char_p, []),
    "mraft_abi_version": (ctypes.c_int, []),
    "mraft_load_state": (ctypes.c_int, [_vp, ctypes.POINTER(MraftSoa), _i32]),
    "mraft_store_state": (ctypes.c_int, [_vp, ctypes.POINTER(MraftSoa), _i32]),
    "mraft_state_view": (ctypes.c_int, [_vp, ctypes.POINTER(MraftSoa)]),
    "mraft_bind_state": (ctypes.c_int, [_vp, ctypes.POINTER(MraftSoa)]),
    "mraft_gather_append_args": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _i32]),
    "mraft_handle_append_entries": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32]),
    "mraft_process_append_replies": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32]),
    "mraft_replicate_tick": (ctypes.c_int, [_vp, _vp, _vp, _i32]),
    "mraft_replicate_tick_count": (ctypes.c_int, [_vp, _vp, _vp, _i32]),
    "mraft_start": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i32]),
    "mraft_collect_apply": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i32]),
    "mraft_election_rounds": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32]),
    "mraft_snapshot": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i32]),
    "mraft_gather_install_snapshot_args": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _i32]),
    "mraft_handle_install_snapshot": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _i32]),
    "mraft_process_install_snapshot_replies": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32]),
    "mraft_start_election": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _i32]),
    "mraft_handle_request_vote": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _i32]),
    "mraft_process_vote_replies": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32]),
    "mraft_export_group_status": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32]),
    "mraft_collect_persist": (ctypes.c_int, [_vp, _vp, _i32]),
    "mraft_read_persistent": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _i64]),
    "mraft_restore": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp]),
    "mraft_encode_persistent": (ctypes.c_int64, [_vp, _vp, _vp, _i64]),
    "mraft_decode_persistent": (ctypes.c_int, [_vp, _i64, _vp, _vp, _i64]),
    "mraft_key2shard": (ctypes.c_int, [ctypes.c_char_p, _i64, _i32]),
    "mraft_replicate_tick_export": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i32]),
    "mraft_collect_apply_compact": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i32]),
    "mraft_realloc_gid": (ctypes.c_int, [_vp, _i32, _vp, _i32]),
    "mraft_comm_unique_id": (ctypes.c_int, [_vp]),
    "mraft_comm_init": (ctypes.c_int, [_vp, _i32, _i32, _vp, ctypes.POINTER(_vp)]),
    "mraft_comm_destroy": (ctypes.c_int, [_vp]),
    "mraft_allgather_status": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _u32]),
    "mraft_fanin_synchronize": (ctypes.c_int, [_vp]),
    "mraft_fanin_stream": (_vp, [_vp]),
    "mraft_fanin_reserve_cus": (ctypes.c_int, [_vp, _i32]),
    "mraft_set_tick_shards": (ctypes.c_int, [_vp, _i32]),
    "mraft_handle_append_entries_ex": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i32]),
    "mraft_get_tick_shards": (_i32, [_vp]),
    "mraft_shard_stream": (_vp, [_vp, _i32]),
    "mraft_set_stage_capacity": (ctypes.c_int, [_vp, _i64]),
    "mraft_get_stage_capacity": (_i64, [_vp]),
    "mraft_set_tick_mode": (ctypes.c_int, [_vp, _i32]),
    "mraft_get_tick_mode": (_i32, [_vp]),
    "mraft_tick_light_fallbacks": (_i64, [_vp]),
    "mraft_start_and_tick": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32]),
}
_SYNTH_SIGS = {
    "mraft_synth_tick_state": (ctypes.c_int, [ctypes.c_uint64, _i32, _i32, _i32, _i32, _i32,
                                              ctypes.POINTER(MraftSoa), _vp, _vp, _i32]),
    "mraft_synth_fold_batch": (ctypes.c_int64, [ctypes.c_uint64, _i32, _i32, _i32,
                                                ctypes.POINTER(MraftSoa), _vp, _vp, _vp]),
    "mraft_synth_election_state": (ctypes.c_int, [ctypes.c_uint64, _i32, _i32, _i32, _i32, _i32,
                                                  ctypes.POINTER(MraftSoa), _vp, _i32, _i32]),
}

_lib = None
_synth = None


def _bind(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)  # AttributeError if not exported: fail loudly
        fn.restype = res
        fn.argtypes = args


def lib():
    """The product library. Raises if it is missing (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with "
                               "`make -C multiraft_amd/csrc` (or __graft_entry__.build())")
        # Share one HIP runtime with torch when torch is present: torch bundles
        # its own libamdhip64.so.7, and the loader dedups by SONAME only if torch
        # is loaded first.
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is plumbing, not required
            pass
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _bind(l, _SIGS)
        _lib = l
    return _lib


def synth():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} is missing: build it with `make -C multiraft_amd/csrc`")
        s = ctypes.CDLL(SYNTH_PATH)
        _bind(s, _SYNTH_SIGS)
        _synth = s
    return _synth


def last_error() -> str:
    return lib().mraft_last_error_string().decode()


def ptr(a) -> int | None:
    """Device or host address of a numpy array / torch tensor (None passes NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    if isinstance(a, int):
        return a
    raise TypeError(type(a))


def soa_of(st: dict) -> MraftSoa:
    s = MraftSoa()
    for f in STATE_FIELDS:
        setattr(s, f, ptr(st.get(f)))
    return s
