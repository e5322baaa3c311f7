"""Per-segment phase timeline of mraft_process_append_replies at config #3
(diagnostic build with -DMRAFT_FOLD_TRACE=1, loaded via MRAFT_LIB): the
message path gather -> handle -> assemble runs first, then the fold with
s_memrealtime stamps (100 MHz) at entry, after the replies arrive, after the
replica state arrives, after the fold arithmetic, after the a1 probes/scans,
and at exit."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    from multiraft_amd import _abi
    from multiraft_amd._abi import AE_RESULT
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    eng = Engine(G, P, L)
    eng.load_state(st)
    slots = np.repeat(np.arange(G) * P + lp, P - 1).astype(np.int32)
    peers = np.array([p for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    args, gerr = eng.gather_append_args(slots, peers)
    rep, herr = eng.handle_append_entries(args, None)
    res = np.zeros(len(slots), dtype=AE_RESULT)
    res["slot"], res["peer"] = slots, peers
    res["args_term"], res["args_prev_log_index"] = args["term"], args["prev_log_index"]
    res["args_n_entries"] = args["n_entries"]
    res["reply_term"], res["reply_success"] = rep["term"], rep["success"]
    res["reply_conflict_index"] = rep["conflict_index"]
    seg = np.arange(0, len(slots) + 1, P - 1, dtype=np.int64)
    f, e = eng.process_append_replies(res, seg)
    torch.cuda.synchronize()
    lib = _abi.lib()
    fn = lib.mraft_debug_fold_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    tr = np.zeros(G * 6, dtype=np.uint64)
    assert fn(tr.ctypes.data, tr.nbytes) == 0
    t = tr.reshape(G, 6).astype(np.int64)
    t -= t[:, 0].min()
    us = t / 100.0
    print(f"span {us[:, 5].max():.1f} us, last start {us[:, 0].max():.1f}, errors {int((e != 0).sum())}")
    names = ("entry->replies", "replies->state", "state->fold done", "a1 probes/scans", "writes")
    for k, name in enumerate(names):
        x = us[:, k + 1] - us[:, k]
        q = np.percentile(x, [10, 50, 90, 99, 100])
        print(f"{name:20s} mean {x.mean():7.2f} p10 {q[0]:6.2f} p50 {q[1]:6.2f} p90 {q[2]:6.2f} "
              f"p99 {q[3]:7.2f} max {q[4]:7.2f} us")
    life = us[:, 5] - us[:, 0]
    print(f"lifetime mean {life.mean():.2f} us; concurrent segments (mean) {life.sum() / us[:, 5].max():.0f}")
    eng.close()


if __name__ == "__main__":
    main()
