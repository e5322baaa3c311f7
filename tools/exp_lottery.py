"""Which part of a state copy decides whether its tick is fast (~0.34 ms) or
slow (~0.38 ms)? (the populations are fixed per allocation.)

For N torch-cloned copies (as bench.py makes them) the tick is timed on
  own      — the copy's own arrays;
  swaplog  — copy i's log_term with copy (i+1)'s scalar/match/next arrays;
  flat     — copy i's log_term with its small arrays re-packed into one
             buffer at skewed (non power-of-two) offsets;
and the addresses are printed, to see whether the slow property follows the
log image or the small arrays (whose 2 MiB-rounded allocations put the
header's same-index reads at power-of-two strides)."""
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
    small = [k for k in master if k != "log_term"]
    # flat re-pack of the small arrays per copy: one buffer, each array at a
    # 4 KiB * (k+1) + 256 B * k skew after the previous one
    flats = []
    for i in range(N):
        sizes = [master[k].numel() for k in small]
        offs, o = [], 0
        for j, n in enumerate(sizes):
            o += (4096 * (j + 1) + 256 * j) // 4
            offs.append(o)
            o += n
        buf = torch.empty(o + 1024, dtype=torch.int32, device=dev)
        flats.append({k: buf[offs[j]:offs[j] + sizes[j]] for j, k in enumerate(small)})
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)

    def timed(state):
        for k in state:
            state[k].copy_(master[k])
        eng.bind(state)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.replicate_tick(lp_d, gf, where=DEVICE)
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    modes = {
        "own": lambda i: clones[i],
        "swaplog": lambda i: {**{k: clones[(i + 1) % N][k] for k in small}, "log_term": clones[i]["log_term"]},
        "flat": lambda i: {**flats[i], "log_term": clones[i]["log_term"]},
    }
    R = 3
    res = {m: np.zeros((N, R)) for m in modes}
    for r in range(R):
        for m, f in modes.items():
            for i in range(N):
                res[m][i, r] = timed(f(i))
    for i in range(N):
        pa = clones[i]["log_term"].data_ptr()
        pt = clones[i]["current_term"].data_ptr()
        print(f"copy {i:2d} log @ {pa:#x} (mod 1G {pa % (1 << 30):#x}) term @ {pt:#x} "
              f"(mod 2M {pt % (1 << 21):#x}) | " +
              " | ".join(f"{m} " + " ".join(f"{x:.3f}" for x in res[m][i]) for m in modes), flush=True)
    for m in modes:
        v = res[m].min(axis=1)
        print(f"{m}: mean of per-copy min {v.mean():.4f} ms, mean {res[m].mean():.4f}, "
              f"fast(<0.36) {int((v < 0.36).sum())}/{N}")
    print("small-array bases (copy 0):", {k: hex(clones[0][k].data_ptr()) for k in small})


if __name__ == "__main__":
    main()
