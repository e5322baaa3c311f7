"""Placement experiment: on N plain (torch / hipMalloc) log images, the tick's time
and the synthetic traffic probe (tools/probe_place.hip) under different
group -> XCD orders: which orders are fast on every image?"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    G, P, L = 65536, 5, 4096
    N = int(os.environ.get("COPIES", 8))
    modes = [int(m) for m in os.environ.get("MODES", "0,1,2,3,4,5,6").split(",")]
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    del st
    probe = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_place.so"))
    probe.probe_place.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    sink = torch.zeros(16, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    small = {k: v.clone() for k, v in master.items() if k != "log_term"}
    imgs = [torch.empty_like(master["log_term"]) for _ in range(N)]  # plain allocations
    print("modes " + " ".join(str(m) for m in modes), flush=True)
    for i, t in enumerate(imgs):
        best = 1e9
        for _ in range(2):
            t.copy_(master["log_term"])
            for k in small:
                small[k].copy_(master[k])
            d = dict(small)
            d["log_term"] = t
            eng.bind(d)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        pr = []
        for m in modes:
            ms = ctypes.c_float()
            assert probe.probe_place(t.data_ptr(), G, P, L, sink.data_ptr(), ctypes.byref(ms), m) == 0
            pr.append(ms.value)
        extra = ""
        if os.environ.get("RANGES", "0") == "1":
            # plain streaming writes over each 1-GiB piece of the image (TB/s)
            probe.probe_write_range.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_float)]
            nbytes, gib, rates = t.numel() * 4, 1 << 30, []
            for off in range(0, nbytes - gib + 1, gib):
                ms = ctypes.c_float()
                assert probe.probe_write_range(t.data_ptr() + off, gib, ctypes.byref(ms)) == 0
                rates.append(gib / (ms.value * 1e-3) / 1e12)
            extra = " | write TB/s per GiB " + " ".join(f"{x:.2f}" for x in rates)
        print(f"image {i}: tick {best:.4f} ms | probe " + " ".join(f"{x:.4f}" for x in pr) + extra, flush=True)
    eng.close()


if __name__ == "__main__":
    main()
