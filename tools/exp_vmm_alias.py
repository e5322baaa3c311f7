"""Placement experiment (the slow/fast state copies): does a
copy's speed follow its PHYSICAL memory or its VIRTUAL addresses?

For each of N copies the log image is backed by physical chunks (hipMemCreate,
CHUNK bytes each) mapped at two virtual ranges: A (chunks in order) and B (the
same chunks in the same order at another address); with SHUFFLE=1 range B maps
the chunks in a permuted order (same physical memory, different VA -> PA
layout). The tick runs through A and through B (log restored from the master
before every run). Same time through A and B = the physical pages decide;
different = the virtual layout (translation) decides."""
import ctypes
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
    del st
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    nbytes = master["log_term"].numel() * 4
    N = int(os.environ.get("COPIES", 6))
    chunk = int(os.environ.get("CHUNK", 1 << 30))
    shuffle = os.environ.get("SHUFFLE", "0") == "1"

    class Loc(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle", ctypes.c_int), ("loc", Loc),
                    ("win32", ctypes.c_void_p), ("cflags", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort), ("_pad", ctypes.c_uint)]

    class Access(ctypes.Structure):
        _fields_ = [("loc", Loc), ("flags", ctypes.c_int)]

    prop = Prop(1, 0, Loc(1, 0), None, 0, 0, 0, 0)
    g = ctypes.c_size_t()
    assert hip.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), 1) == 0
    gran = max(g.value, chunk)
    size = (nbytes + gran - 1) // gran * gran
    nch = size // gran

    def reserve():
        va = ctypes.c_void_p()
        rc = hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(size), ctypes.c_size_t(gran), None,
                                      ctypes.c_ulonglong(0))
        assert rc == 0, rc
        return va.value

    def map_at(va, handles, order):
        for slot, k in enumerate(order):
            rc = hip.hipMemMap(ctypes.c_void_p(va + slot * gran), ctypes.c_size_t(gran), ctypes.c_size_t(0),
                               handles[k], ctypes.c_ulonglong(0))
            assert rc == 0, rc
        acc = Access(Loc(1, 0), 3)
        assert hip.hipMemSetAccess(ctypes.c_void_p(va), ctypes.c_size_t(size), ctypes.byref(acc),
                                   ctypes.c_size_t(1)) == 0

    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    small = {k: v.clone() for k, v in master.items() if k != "log_term"}
    rng = np.random.default_rng(1)
    print(f"chunk {gran} B x {nch} per copy, shuffle={shuffle}", flush=True)
    copies = []
    for i in range(N):
        handles = []
        for _ in range(nch):
            h = ctypes.c_void_p()
            assert hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(gran), ctypes.byref(prop),
                                    ctypes.c_ulonglong(0)) == 0
            handles.append(h)
        va_a, va_b = reserve(), reserve()
        map_at(va_a, handles, list(range(nch)))
        order_b = list(rng.permutation(nch)) if shuffle else list(range(nch))
        map_at(va_b, handles, order_b)
        copies.append((va_a, va_b, order_b))

    def run(p):
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
        return a.elapsed_time(b)

    for rep in range(2):
        for i, (va_a, va_b, order_b) in enumerate(copies):
            ta = min(run(va_a) for _ in range(2))
            tb = min(run(va_b) for _ in range(2))
            print(f"rep {rep} copy {i}: A {ta:.4f} ms @ {va_a:#x}   B {tb:.4f} ms @ {va_b:#x}"
                  + (f" order {order_b}" if shuffle else ""), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
