"""Are the two step-time populations (≈0.35 / ≈0.39 ms) a property of the
state copy (its allocation) or of time? Runs every copy several times,
restoring its content in between, and prints the tick time per copy with the
log_term address."""
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
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    times = np.zeros((N, 3))
    for r in range(3):
        for i, c in enumerate(clones):
            for k in c:
                c[k].copy_(master[k])
            eng.bind(c)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            times[i, r] = a.elapsed_time(b)
    for i, c in enumerate(clones):
        pa = c["log_term"].data_ptr()
        print(f"copy {i:2d} log_term @ {pa:#x} (mod 1GiB {pa % (1 << 30):#x}) ms " +
              " ".join(f"{x:.3f}" for x in times[i]))


if __name__ == "__main__":
    main()
