"""Does the row stride decide the slow population? A wave
compares / copies the leader's and up to four followers' rows at the SAME
entry offset, i.e. at addresses 16 KiB apart (L = 4,096). For each row
padding (capacity L + pad, same logs and algorithmic words), N fresh copies
are timed; prints per-pad copy times."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("COPIES", 8))
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    for pad in [int(x) for x in os.environ.get("PADS", "0,1024,2048,96").split(",")]:
        s2 = dict(st)
        if pad:
            s2["log_term"] = np.ascontiguousarray(np.pad(st["log_term"].reshape(G * P, L), ((0, 0), (0, pad))).reshape(-1))
        master = {k: torch.from_numpy(v).to(dev) for k, v in s2.items()}
        clones = [{k: v.clone() for k, v in master.items()} for _ in range(N)]
        eng = Engine(G, P, L + pad, alloc=False)
        eng.set_stream(stream.cuda_stream)
        t = np.zeros((N, 2))
        for r in range(2):
            for i, c in enumerate(clones):
                for k in c:
                    c[k].copy_(master[k])
                eng.bind(c)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                eng.replicate_tick(lp_d, gf, where=DEVICE)
                b.record(stream)
                torch.cuda.synchronize()
                t[i, r] = a.elapsed_time(b)
        m = t.min(axis=1)
        print(f"pad {pad}: copies " + " ".join(f"{x:.3f}" for x in m) + f" | mean {m.mean():.4f} "
              f"slow(>0.36) {int((m > 0.36).sum())}/{N}", flush=True)
        eng.close()
        del clones, master
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
