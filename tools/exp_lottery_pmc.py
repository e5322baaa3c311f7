"""PMC companion of exp_lottery.py: one tick per copy (two passes, the copy
restored before each), printed with its time, so a rocprofv3 --pmc run over
this script gives per-copy counters (dispatch order = copy order) for fast
and slow copies of the log image."""
import os
import sys

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
            print(f"pass {r} copy {i} ms {a.elapsed_time(b):.4f} log {c['log_term'].data_ptr():#x}", flush=True)


if __name__ == "__main__":
    main()
