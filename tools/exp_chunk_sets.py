"""Placement experiment, continued (tools/exp_chunk_probe.py: a log image
assembled from 1-GiB chunks of DIFFERENT allocations runs fast, five chunks
allocated back to back mostly run slow): which sets of physical chunks make
a fast image?

One pool of POOL chunks of CHUNK bytes (hipMemCreate, allocated back to back);
each image named in IMAGES ("0,1,2,3,4;0,2,4,6,8;...": pool indices, in VA
order) is mapped and the tick timed on it (best of 2, log restored first)."""
import ctypes
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
    del st
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    nbytes = master["log_term"].numel() * 4
    gran = int(os.environ.get("CHUNK", 1 << 30))
    pool_n = int(os.environ.get("POOL", 12))
    nch = (nbytes + gran - 1) // gran
    images = [[int(x) for x in s.split(",")] for s in os.environ["IMAGES"].split(";")]

    class Loc(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle", ctypes.c_int), ("loc", Loc),
                    ("win32", ctypes.c_void_p), ("cflags", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort), ("_pad", ctypes.c_uint)]

    class Access(ctypes.Structure):
        _fields_ = [("loc", Loc), ("flags", ctypes.c_int)]

    prop = Prop(1, 0, Loc(1, 0), None, 0, 0, 0, 0)
    pool = []
    for _ in range(pool_n):
        h = ctypes.c_void_p()
        assert hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(gran), ctypes.byref(prop), ctypes.c_ulonglong(0)) == 0
        pool.append(h)

    def image(idx):
        assert len(idx) == nch, (len(idx), nch)
        va = ctypes.c_void_p()
        assert hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(nch * gran), ctypes.c_size_t(gran), None,
                                        ctypes.c_ulonglong(0)) == 0
        for k, j in enumerate(idx):
            assert hip.hipMemMap(ctypes.c_void_p(va.value + k * gran), ctypes.c_size_t(gran), ctypes.c_size_t(0),
                                 pool[j], ctypes.c_ulonglong(0)) == 0
        acc = Access(Loc(1, 0), 3)
        assert hip.hipMemSetAccess(va, ctypes.c_size_t(nch * gran), ctypes.byref(acc), ctypes.c_size_t(1)) == 0
        return va.value

    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    small = {k: v.clone() for k, v in master.items() if k != "log_term"}

    def tick(p):
        best = 1e9
        for _ in range(2):
            torch.cuda.synchronize()
            assert hip.hipMemcpy(p, master["log_term"].data_ptr(), nbytes, 3) == 0
            for k in small:
                small[k].copy_(master[k])
            torch.cuda.synchronize()
            d = dict(small)
            d["log_term"] = p
            eng.bind(d)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        return best

    probe = None
    if os.environ.get("PROBE", "0") == "1":
        probe = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_place.so"))
        probe.probe_place.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_float)]
        sink = torch.zeros(16, dtype=torch.int32, device=dev)
    print(f"pool of {pool_n} chunks of {gran} B; {nch} per image", flush=True)
    for idx in images:
        va = image(idx)
        t = tick(va)
        extra = ""
        if probe is not None:
            torch.cuda.synchronize()
            ms = ctypes.c_float()
            assert probe.probe_place(va, G, P, L, sink.data_ptr(), ctypes.byref(ms)) == 0
            extra = f"  probe {ms.value:.4f} ms"
        print(f"image {idx}: tick {t:.4f} ms{extra}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
