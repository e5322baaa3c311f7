"""Second placement experiment: is the slow tick population
the state the caches are left in by the preceding work? Per copy: restore,
then (a) tick at once, (b) read a 2 GiB unrelated buffer first (evicts and
writes back the L2 / Infinity-Cache lines the restore dirtied), (c) sleep
50 ms on the host first, (d) write-read-write: restore, flush, restore again."""
import os
import sys
import time

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
    junk = torch.ones(512 * 1024 * 1024, dtype=torch.int32, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)

    def tick():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.replicate_tick(lp_d, gf, where=DEVICE)
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    def restore(c):
        for k in c:
            c[k].copy_(master[k])

    def flush():
        sink.add_(junk.sum())

    variants = {
        "a_direct": lambda c: (restore(c), None),
        "b_flush": lambda c: (restore(c), flush()),
        "c_sleep": lambda c: (restore(c), torch.cuda.synchronize(), time.sleep(0.05)),
        "d_flush_sleep": lambda c: (restore(c), flush(), torch.cuda.synchronize(), time.sleep(0.05)),
    }
    res = {v: np.zeros((N, 2)) for v in variants}
    for r in range(2):
        for v, prep in variants.items():
            for i, c in enumerate(clones):
                prep(c)
                eng.bind(c)
                res[v][i, r] = tick()
    for i in range(N):
        print(f"copy {i:2d} " + " | ".join(f"{v} " + " ".join(f"{x:.3f}" for x in res[v][i]) for v in variants),
              flush=True)
    for v in variants:
        print(f"{v}: mean {res[v].mean():.4f} min-of-copy mean {res[v].min(axis=1).mean():.4f} "
              f"slow(>0.36) {int((res[v] > 0.36).sum())}/{res[v].size}")


if __name__ == "__main__":
    main()
