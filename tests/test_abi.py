"""CPU checks of the boundary: the shared library loads without a GPU and
exports every symbol include/mraft.h declares (no compute calls)."""
import ctypes
import os
import re

import pytest

from multiraft_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return set(re.findall(r"^\s*(?:int|int32_t|int64_t|void\s*\*|const char\s*\*)\s*\*?\s*(mraft_\w+)\s*\(",
                          txt, re.M))


def test_header_symbols_match_binding_list():
    assert _declared("mraft.h") == set(_abi.ABI_SYMBOLS)
    assert _declared("mraft_synth.h") == set(_abi.SYNTH_SYMBOLS)


def test_library_exports_every_symbol():
    assert os.path.exists(_abi.LIB_PATH), "build libmraft_hip.so first"
    lib = ctypes.CDLL(_abi.LIB_PATH)
    for s in _abi.ABI_SYMBOLS:
        assert hasattr(lib, s), s
    syn = ctypes.CDLL(_abi.SYNTH_PATH)
    for s in _abi.SYNTH_SYMBOLS:
        assert hasattr(syn, s), s


def test_abi_version_and_struct_sizes():
    lib = _abi.lib()
    assert lib.mraft_abi_version() == _abi.ABI_VERSION == 6
    assert _abi.AE_ARGS.itemsize == 40
    assert _abi.AE_REPLY.itemsize == 16
    assert _abi.RV_RESULT.itemsize == 20
    assert ctypes.sizeof(_abi.MraftSoa) == 15 * 8
    assert _abi.PERSISTENT.itemsize == 32


def test_create_rejects_bad_dims_without_gpu():
    lib = _abi.lib()
    h = ctypes.c_void_p()
    assert lib.mraft_create(0, 5, 16, 0, 0, ctypes.byref(h)) == _abi.E_INVAL
    assert lib.mraft_create(4, 9, 16, 0, 0, ctypes.byref(h)) == _abi.E_INVAL
    assert b"bad dims" in lib.mraft_last_error_string()


def test_persistent_codec_round_trip_host_only():
    """mraft_encode_persistent / mraft_decode_persistent are host code: they
    run without a GPU. Round trip, exact size, and malformed-buffer rejection."""
    import numpy as np
    from multiraft_amd import decode_persistent, encode_persistent
    from multiraft_amd.engine import MraftError
    rec = {"current_term": 7, "voted_for": -1, "dummy_index": 40, "last_index": 44}
    terms = np.array([3, 3, 5, 7, 7], np.int32)
    b = encode_persistent(rec, terms)
    assert len(b) == 36 + 8 * 5 and b[:4] == b"MRPS"
    r, t = decode_persistent(b)
    assert (int(r["current_term"]), int(r["voted_for"]), int(r["dummy_index"]),
            int(r["last_index"])) == (7, -1, 40, 44)
    assert t.tolist() == terms.tolist()
    for bad in (b[:-1], b"XRPS" + b[4:], b[:32] + (6).to_bytes(4, "little") + b[36:]):
        try:
            decode_persistent(bad)
        except MraftError:
            continue
        raise AssertionError("malformed buffer accepted")


@pytest.mark.gpu
def test_message_calls_reject_bad_arguments_gpu():
    """The message-path entry points check their arguments before any launch:
    a negative item count, a null output, a negative entry-word count with a
    caller buffer, n_seg < 0, a stage capacity outside [0, 2^31) — each
    MRAFT_E_INVAL with a message, and the engine ticks on afterwards."""
    import numpy as np
    from oracle_lib import Oracle, assert_states_equal
    from multiraft_amd import Engine, synth_tick_state
    from multiraft_amd._abi import AE_ARGS, AE_REPLY, AE_RESULT, HOST, ptr
    lib = _abi.lib()
    G, P, L = 8, 3, 16
    st, lp, _ = synth_tick_state(G, P, L, seed=7)
    a, r, err = np.zeros(2, AE_ARGS), np.zeros(2, AE_REPLY), np.zeros(2, np.int32)
    terms = np.zeros(4, np.int32)
    res, fl, seg = np.zeros(2, AE_RESULT), np.zeros(2, np.int32), np.zeros(3, np.int64)
    with Engine(G, P, L) as e:
        e.load_state(st)
        h = e._h
        assert lib.mraft_handle_append_entries_ex(h, ptr(a), -1, None, 0, ptr(r), None, ptr(err), HOST) == _abi.E_INVAL
        assert lib.mraft_handle_append_entries_ex(h, ptr(a), 2, None, 0, None, None, ptr(err), HOST) == _abi.E_INVAL
        assert b"null argument" in lib.mraft_last_error_string()
        assert lib.mraft_handle_append_entries_ex(h, ptr(a), 2, ptr(terms), -4, ptr(r), None, ptr(err),
                                                  HOST) == _abi.E_INVAL
        assert b"n_entry_terms" in lib.mraft_last_error_string()
        assert lib.mraft_process_append_replies(h, ptr(res), 2, ptr(seg), -1, ptr(fl), ptr(err), HOST) == _abi.E_INVAL
        assert lib.mraft_process_append_replies(h, ptr(res), -2, None, 0, ptr(fl), ptr(err), HOST) == _abi.E_INVAL
        assert lib.mraft_set_stage_capacity(h, -2) == _abi.E_INVAL
        assert lib.mraft_set_stage_capacity(h, 1 << 31) == _abi.E_INVAL
        assert lib.mraft_get_stage_capacity(h) == 4 << 20  # unchanged default
        assert lib.mraft_set_stage_capacity(h, -1) == 0  # MRAFT_STAGE_AUTO (the default mode)
        assert lib.mraft_get_stage_capacity(h) == 4 << 20
        gf = e.replicate_tick(lp)
        o = Oracle(G, P, L, st)
        assert np.array_equal(gf, o.replicate_tick(lp))
        assert_states_equal(e.store_state(), o.state(), G, P, L, "after rejected calls")
