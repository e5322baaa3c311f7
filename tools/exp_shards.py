"""Experiment: config #3's 65,536 groups as S independent shards, one engine
and one stream each, ticked in turn every step (shard s's tick i+1 follows its
tick i on its own stream; the shards' launches overlap across streams), so one
launch's last generation of groups shares the device with the next launch's
first. Same workload per step as bench.py (every group ticks once, fresh state
copy per step); whole-step wall time over K steps, and the shards' flags and
export words checked against the one-engine tick.

Env: SHARDS (e.g. "1,2,4"), STEPS, REPS, GROUPS_TOTAL."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    S_list = [int(x) for x in os.environ.get("SHARDS", "1,2,4").split(",")]
    G = int(os.environ.get("GROUPS_TOTAL", 65536))
    P, L = 5, 4096
    K = int(os.environ.get("STEPS", 16))
    dev = torch.device("cuda", 0)
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=16)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    per = {k: v.numel() // G for k, v in master.items()}
    del st
    # the SAME physical copies for every shard count (the placement lottery,
    # DESIGN.md §5, is then common to all variants); restored between runs
    copies = [{k: v.clone() for k, v in master.items()} for _ in range(K)]
    lp_d = torch.from_numpy(lp).to(dev)
    outs = {k: torch.zeros(G, dtype=torch.int32, device=dev) for k in ("gf", "cm", "tl")}

    def part(d, s, g):
        return {k: v[s * g * per[k]:(s + 1) * g * per[k]] for k, v in d.items()}

    setups = {}
    for S in S_list:
        g = G // S
        sh = []
        for s in range(S):
            stream = torch.cuda.Stream(dev)
            eng = Engine(g, P, L, device=0, alloc=False)
            eng.set_stream(stream.cuda_stream)
            sh.append((eng, stream, lp_d[s * g:(s + 1) * g], {k: v[s * g:(s + 1) * g] for k, v in outs.items()}))
        setups[S] = (g, sh)
    ref = None
    res = {S: [] for S in S_list}
    for rep in range(int(os.environ.get("REPS", 3))):
        for S in S_list:
            g, sh = setups[S]
            parts = [[part(copies[i], s, g) for s in range(S)] for i in range(K)]  # host work outside the timing
            for c in copies:
                for k in c:
                    c[k].copy_(master[k])
            for v in outs.values():
                v.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                for s, (eng, stream, lps, o) in enumerate(sh):
                    eng.bind(parts[i][s])
                    eng.replicate_tick_export(lps, o["gf"], o["cm"], o["tl"], where=DEVICE)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            out = [outs[k].cpu().numpy() for k in ("gf", "cm", "tl")]
            if ref is None:
                ref = out
            same = all(np.array_equal(a, b) for a, b in zip(out, ref))
            res[S].append(dt / K * 1e3)
            print(json.dumps({"shards": S, "rep": rep, "ms_per_step": dt / K * 1e3, "equal_to_first": same}),
                  flush=True)
            assert same
    print(json.dumps({"summary": {S: {"mean": float(np.mean(v)), "min": float(np.min(v))} for S, v in res.items()}}))


if __name__ == "__main__":
    main()
