"""Per-group phase timeline of the headline tick (diagnostic build with
-DMRAFT_TICK_TRACE=1, loaded via MRAFT_LIB): s_memrealtime stamps (100 MHz)
at entry, before the streaming pass, after it, and at exit. Prints phase
duration percentiles and how many groups are inside each phase over time."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    from multiraft_amd import _abi
    G, P, L = int(os.environ.get("TRACE_G", 65536)), 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(3)]
    eng = Engine(G, P, L, alloc=False)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    lib = _abi.lib()
    fn = lib.mraft_debug_tick_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    for i, c in enumerate(clones):
        eng.bind(c)
        eng.replicate_tick(lp_d, gf, where=DEVICE)
        torch.cuda.synchronize()
    tr = np.zeros(G * 4, dtype=np.uint64)
    assert fn(tr.ctypes.data, tr.nbytes) == 0
    tr = tr.reshape(G, 4)
    xcc = (tr[:, 0] >> np.uint64(60)).astype(np.int64)   # the entry stamp carries the XCD in its top bits
    t = (tr & np.uint64((1 << 60) - 1)).astype(np.int64)
    t -= t[:, 0].min()
    us = t / 100.0  # 100 MHz -> us
    if os.environ.get("TRACE_SAVE"):
        np.save(os.environ["TRACE_SAVE"], np.concatenate([us, xcc[:, None]], axis=1))
    hdr, pas, tail, life = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2], us[:, 3] - us[:, 0]
    span = us[:, 3].max()
    print(f"span {span:.1f} us (first start {us[:,0].min():.1f}, last start {us[:,0].max():.1f}, "
          f"first end {us[:,3].min():.1f})")
    for name, x in (("header+A+scans", hdr), ("pass", pas), ("C+D", tail), ("lifetime", life)):
        q = np.percentile(x, [10, 50, 90, 99, 100])
        print(f"{name:15s} mean {x.mean():7.2f}  p10 {q[0]:6.2f} p50 {q[1]:6.2f} p90 {q[2]:6.2f} "
              f"p99 {q[3]:7.2f} max {q[4]:7.2f} us")
    print(f"sum over groups: header {hdr.sum()/1e3:.1f} ms, pass {pas.sum()/1e3:.1f} ms, C+D {tail.sum()/1e3:.1f} ms")
    # The ramp-down: who finishes last, when they started, how long they lived.
    end = us[:, 3]
    for frac in (0.001, 0.01, 0.05):
        k = max(1, int(G * frac))
        idx = np.argsort(end)[-k:]
        print(f"last {frac*100:.1f}% to finish ({k} groups): end >= {end[idx].min():.1f} us, start p10/p50/p90 "
              f"{np.percentile(us[idx, 0], 10):.1f}/{np.percentile(us[idx, 0], 50):.1f}/{np.percentile(us[idx, 0], 90):.1f}, "
              f"lifetime p50 {np.median(life[idx]):.1f} (all groups p50 {np.median(life):.1f}), pass p50 {np.median(pas[idx]):.1f}")
    grid = np.arange(0, span + 5, 5.0)
    print(" t(us)  in-header  in-pass  in-CD  done")
    for x in grid:
        a = ((us[:, 0] <= x) & (us[:, 1] > x)).sum()
        b = ((us[:, 1] <= x) & (us[:, 2] > x)).sum()
        c = ((us[:, 2] <= x) & (us[:, 3] > x)).sum()
        d = (us[:, 3] <= x).sum()
        print(f"{x:6.0f} {a:9d} {b:8d} {c:6d} {d:6d}")
    eng.close()


if __name__ == "__main__":
    main()
