"""Diagnostic: the deferred items' pass records (MRAFT_AE_DBG variant) for the rows that differ."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["MRAFT_LIB"] = os.path.join(ROOT, "tools/variants/libmraft_hip_dbg.so")
from message_cases import stale_cycle_state  # noqa: E402
from oracle_lib import Oracle, logical_logs  # noqa: E402

from multiraft_amd import Engine, synth_tick_state  # noqa: E402

lib = ctypes.CDLL(os.environ["MRAFT_LIB"])
buf = np.zeros((4096, 32), np.int32)
G, P, L = 256, 5, 128
names = "slot plo phi cfrom vec flat src0 src64 pre0 pre64 post0 post64 mode so start cend pren pref postn postf c copy cmp x dcalls dc0 passv passn dact de22 di22 dk".split()
for cap in (0, None, None):
    rng = np.random.default_rng(18)
    st, lp, _ = synth_tick_state(G, P, L, seed=78)
    st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(0, G, 3), 2)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap is not None:
            e.set_stage_capacity(cap)
        args, gerr = e.gather_append_args(slots, peers)
        batch = args[gerr == 0]
        lib.mraft_debug_aedbg(buf.ctypes.data_as(ctypes.c_void_p), 4096)
        rep, herr = e.handle_append_entries(batch, None)
        nrec = lib.mraft_debug_aedbg(buf.ctypes.data_as(ctypes.c_void_p), 4096)
        orep, oherr = o.handle_append_entries(batch, None)
        g, w = e.store_state(), o.state()
    lg, lw = logical_logs(g, G, P, L), logical_logs(w, G, P, L)
    live = w["last_index"] - w["dummy_index"]
    bad = [r for r in range(G * P) if not np.array_equal(lg[r, :live[r] + 1], lw[r, :live[r] + 1])]
    print(f"cap {cap}: {nrec} records, bad rows {bad}")
    recs = buf[:nrec]
    for r in bad:
        for rec in recs[recs[:, 0] == r]:
            print("   ", " ".join(f"{k}={v}" for k, v in zip(names, rec)))
    if cap == 0:
        for rec in recs:
            print("  all", " ".join(f"{k}={v}" for k, v in zip(names, rec) if k in ("slot", "plo", "phi", "vec", "so", "c", "x", "pren", "postn", "g0", "g1", "g2", "g3", "plain", "nt", "widx", "lineoff", "src64")),
                  "src", int(batch[rec[23]]["entries_offset"]) // L, "prev", int(batch[rec[23]]["prev_log_index"]))
    # and a few good ones of the same shape for comparison
    good = [rec for rec in recs if rec[0] not in bad and rec[5] == 1][:3]
    for rec in good:
        print("  ok", " ".join(f"{k}={v}" for k, v in zip(names, rec)))
