"""Per-XCD view of the placement lottery: runs the headline
tick on N fresh state copies with a diagnostic build (-DMRAFT_TICK_TRACE=1,
loaded via MRAFT_LIB) and, per copy, prints the launch time and for each XCD
(hardware XCC id stamped by the wave) its group count, when its last group
ended, and its mean pass duration. A copy that is slow because one XCD's
range of the log image is slow shows one late XCD; a uniformly slow copy
shows all eight late."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    from multiraft_amd import _abi
    G, P, L = 65536, 5, 4096
    N = int(os.environ.get("COPIES", 8))
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    del st
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(N)]
    eng = Engine(G, P, L, alloc=False)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    fn = _abi.lib().mraft_debug_tick_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    for rep in range(2):
        for i, c in enumerate(clones):
            for k in c:
                c[k].copy_(master[k])
            eng.bind(c)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            tr = np.zeros(G * 4, dtype=np.uint64)
            assert fn(tr.ctypes.data, tr.nbytes) == 0
            t = tr.reshape(G, 4)
            xcc = (t[:, 0] >> np.uint64(60)).astype(np.int64)
            t = (t & np.uint64((1 << 60) - 1)).astype(np.int64)
            t -= t[:, 0].min()
            us = t / 100.0
            parts = []
            for x in range(8):
                m = xcc == x
                if not m.any():
                    continue
                parts.append(f"x{x}:{int(m.sum())}g end {us[m, 3].max():6.1f} pass {np.mean(us[m, 2] - us[m, 1]):5.2f}")
            rng = [f"{us[r * (G // 8):(r + 1) * (G // 8), 3].max():.0f}" for r in range(8)]
            print(f"rep {rep} copy {i}: {ms:.4f} ms span {us[:, 3].max():6.1f} | " + " | ".join(parts)
                  + " | range ends " + ",".join(rng), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
