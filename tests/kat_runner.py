"""Runs the committed KATs (tests/golden/kat.json) through any object with the
Engine interface (the GPU engine, or the CPU oracle wrapper)."""
from __future__ import annotations

import json
import os

import numpy as np

from multiraft_amd._abi import AE_ARGS, AE_RESULT, IS_ARGS, IS_RESULT, RV_ARGS, RV_RESULT

HERE = os.path.dirname(os.path.abspath(__file__))


def load_kats():
    with open(os.path.join(HERE, "golden", "kat.json")) as f:
        return json.load(f)


def kat_state(k):
    st = {kk: np.array(v, dtype=np.int32) for kk, v in k["state"].items()}
    st.setdefault("persist_dirty", np.zeros(k["G"] * k["P"], np.int32))
    st.setdefault("log_head", np.zeros(k["G"] * k["P"], np.int32))
    st.setdefault("has_snapshot", np.zeros(k["G"] * k["P"], np.int32))
    return st


def _rec(dtype, rows):
    a = np.zeros(len(rows), dtype=dtype)
    for i, r in enumerate(rows):
        for f, v in r.items():
            if f == "_pad" and f not in dtype.names:  # fixtures written before AE args carried `flags`
                f = "flags"
            a[f][i] = v
    return a


def run_kat(k, eng, store):
    """eng: engine-like object already holding kat_state(k); store(): returns
    the state dict after the call."""
    out = {}
    if k["op"] == "process_append_replies":
        flags, err = eng.process_append_replies(_rec(AE_RESULT, k["items"]))
        assert not err.any(), err
        out["flags"] = flags.tolist()
    elif k["op"] == "handle_append_entries":
        rep, err = eng.handle_append_entries(_rec(AE_ARGS, k["args"]),
                                             np.array(k["entry_terms"], dtype=np.int32))
        assert not err.any(), err
        out["reply"] = dict(term=int(rep["term"][0]), success=int(rep["success"][0]),
                            conflict_index=int(rep["conflict_index"][0]))
    elif k["op"] == "handle_request_vote":
        rep, err = eng.handle_request_vote(_rec(RV_ARGS, k["args"]))
        assert not err.any(), err
        out["reply"] = dict(term=int(rep["term"][0]), vote_granted=int(rep["vote_granted"][0]))
    elif k["op"] == "process_vote_replies":
        flags, err = eng.process_vote_replies(_rec(RV_RESULT, k["items"]),
                                              np.array([0, len(k["items"])], dtype=np.int64))
        assert not err.any(), err
        out["flags"] = flags.tolist()
    elif k["op"] == "handle_install_snapshot":
        rep, _, err = eng.handle_install_snapshot(_rec(IS_ARGS, k["args"]))
        assert not err.any(), err
        out["is_reply"] = int(rep["term"][0])
    elif k["op"] == "snapshot":
        err = eng.snapshot(np.array(k["slots"], np.int32), np.array(k["index"], np.int32))
        assert not err.any(), err
    elif k["op"] == "start":
        idx, term, isl, err = eng.start(np.array(k["slots"], np.int32))
        assert not err.any(), err
        out["start"] = [[int(a), int(b), int(c)] for a, b, c in zip(idx, term, isl)]
    elif k["op"] == "process_install_snapshot_replies":
        flags, err = eng.process_install_snapshot_replies(
            _rec(IS_RESULT, k["items"]), np.array([0, len(k["items"])], dtype=np.int64))
        assert not err.any(), err
        out["flags"] = flags.tolist()
    out["state"] = store()
    return out
