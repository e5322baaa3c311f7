"""Third placement experiment: do the slow copies depend on
how many waves stream at once? Per copy, the tick at full occupancy, with
fewer waves per CU (dynamic LDS per workgroup: MRAFT_TICK_DYN_LDS, read once
per process, so one process per setting) and on fewer CUs (a CU-masked
stream). Prints one line per copy: the setting's times."""
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
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    N = int(os.environ.get("COPIES", 12))
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(N)]
    eng = Engine(G, P, L, alloc=False)
    cus = [int(x) for x in os.environ.get("MASKS", "0,32,64,128").split(",")]
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    res = np.zeros((len(cus), N, 2))
    for ci, reserve in enumerate(cus):
        eng.fanin_reserve_cus(reserve)  # the tick's stream leaves `reserve` CUs out
        stream = torch.cuda.ExternalStream(eng.stream(), device=dev) if reserve else torch.cuda.Stream(dev)
        if not reserve:
            eng.set_stream(stream.cuda_stream)
        torch.cuda.set_stream(stream)
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
                res[ci, i, r] = a.elapsed_time(b)
    lds = os.environ.get("MRAFT_TICK_DYN_LDS", "0")
    for i in range(N):
        print(f"lds {lds} copy {i:2d} " + " | ".join(f"cus-{c} " + " ".join(f"{x:.3f}" for x in res[ci, i])
                                                  for ci, c in enumerate(cus)), flush=True)
    for ci, c in enumerate(cus):
        print(f"lds {lds} cus-{c}: mean {res[ci].mean():.4f} slow(>0.36) {int((res[ci] > 0.36).sum())}/{res[ci].size}")


if __name__ == "__main__":
    main()
