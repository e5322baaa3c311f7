"""Placement experiment, continued (tools/exp_vmm_alias.py: a state copy's
speed follows its physical memory): per 1-GiB physical chunk, does a plain
streaming copy show the same slow/fast split as the tick?

N copies of the log image, each on 5 hipMemCreate chunks of 1 GiB mapped in
order; for each copy: the tick's time, then per chunk the time of a torch
copy of its first half into its second half (a streaming read + write), and
MIX=1 adds images assembled from chunk k of copy (k + j) mod N."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Arr:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes // 4,), "typestr": "<i4", "data": (ptr, False),
                                         "version": 2}


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
    N = int(os.environ.get("COPIES", 6))
    gran = 1 << 30
    nch = (nbytes + gran - 1) // gran

    class Loc(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle", ctypes.c_int), ("loc", Loc),
                    ("win32", ctypes.c_void_p), ("cflags", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort), ("_pad", ctypes.c_uint)]

    class Access(ctypes.Structure):
        _fields_ = [("loc", Loc), ("flags", ctypes.c_int)]

    prop = Prop(1, 0, Loc(1, 0), None, 0, 0, 0, 0)
    handles = []
    for _ in range(N * nch):
        h = ctypes.c_void_p()
        assert hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(gran), ctypes.byref(prop), ctypes.c_ulonglong(0)) == 0
        handles.append(h)

    def image(hs):
        va = ctypes.c_void_p()
        assert hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(nch * gran), ctypes.c_size_t(gran), None,
                                        ctypes.c_ulonglong(0)) == 0
        for k, h in enumerate(hs):
            assert hip.hipMemMap(ctypes.c_void_p(va.value + k * gran), ctypes.c_size_t(gran), ctypes.c_size_t(0), h,
                                 ctypes.c_ulonglong(0)) == 0
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

    def ev():
        return torch.cuda.Event(enable_timing=True)

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
            a, b = ev(), ev()
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        return best

    def chunk_copy(p):
        t = torch.as_tensor(_Arr(p, gran), device=dev)
        h = t.numel() // 2
        best = 1e9
        for _ in range(3):
            a, b = ev(), ev()
            a.record(stream)
            t[h:].copy_(t[:h])
            b.record(stream)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        return gran / (best * 1e-3) / 1e12  # read + write bytes per s, TB/s

    imgs = [image(handles[i * nch:(i + 1) * nch]) for i in range(N)]
    for i, va in enumerate(imgs):
        t = tick(va)
        bw = [chunk_copy(va + k * gran) for k in range(nch)]
        print(f"copy {i}: tick {t:.4f} ms | chunk copy TB/s " + " ".join(f"{x:.2f}" for x in bw), flush=True)
    if os.environ.get("MIX", "1") == "1":
        for j in range(1, min(N, 4)):
            hs = [handles[((k + j) % N) * nch + k] for k in range(nch)]
            va = image(hs)
            srcs = [(k + j) % N for k in range(nch)]
            print(f"mixed image {j} (chunk k from copy {srcs}): tick {tick(va):.4f} ms", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
