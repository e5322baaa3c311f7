"""Placement experiment: the tick's time on log_term images allocated with
hipExtMallocWithFlags(hipDeviceMallocContiguous) vs plain hipMalloc."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    from multiraft_amd import _abi
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    nbytes = master["log_term"].numel() * 4
    N = int(os.environ.get("COPIES", 3))

    class Loc(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle", ctypes.c_int), ("loc", Loc),
                    ("win32", ctypes.c_void_p), ("cflags", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort), ("_pad", ctypes.c_uint)]

    class Access(ctypes.Structure):
        _fields_ = [("loc", Loc), ("flags", ctypes.c_int)]

    def vmm(chunk_gran):
        """hipMemCreate + hipMemMap: physical chunks of `gran` bytes (or the
        recommended granularity) mapped into one VA range."""
        prop = Prop(1, 0, Loc(1, 0), None, 0, 0, 0, 0)
        g = ctypes.c_size_t()
        assert hip.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), 1) == 0
        gran = max(g.value, chunk_gran or g.value)
        size = (nbytes + gran - 1) // gran * gran
        va = ctypes.c_void_p()
        rc = hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(size), ctypes.c_size_t(gran), None, ctypes.c_ulonglong(0))
        if rc:
            return rc, None
        off = 0
        while off < size:
            h = ctypes.c_void_p()
            rc = hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(gran), ctypes.byref(prop), ctypes.c_ulonglong(0))
            if rc:
                return rc, None
            rc = hip.hipMemMap(ctypes.c_void_p(va.value + off), ctypes.c_size_t(gran), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0))
            if rc:
                return rc, None
            off += gran
        acc = Access(Loc(1, 0), 3)
        rc = hip.hipMemSetAccess(va, ctypes.c_size_t(size), ctypes.byref(acc), ctypes.c_size_t(1))
        print(f"vmm granularity {gran} (recommended {g.value})", flush=True)
        return rc, va.value

    bufs = []
    for kind in os.environ.get("KINDS", "0,vmm,vmm1g,0").split(","):
        for _ in range(N):
            if kind.startswith("vmm"):
                rc, p = vmm(1 << 30 if kind == "vmm1g" else 2 << 20)
                bufs.append((kind, rc, p))
            else:
                p = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, int(kind))
                bufs.append((kind, rc, p.value))
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    small = {k: v.clone() for k, v in master.items() if k != "log_term"}
    for flag, rc, p in bufs:
        if rc != 0:
            print(f"flag {flag}: alloc failed rc={rc}")
            continue
        ts = []
        for r in range(3):
            torch.cuda.synchronize()
            assert hip.hipMemcpy(p, master["log_term"].data_ptr(), nbytes, 3) == 0
            for k in small:
                small[k].copy_(master[k])
            torch.cuda.synchronize()
            assert hip.hipDeviceSynchronize() == 0
            d = dict(small)
            d["log_term"] = p
            eng.bind(d)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            b.record(stream)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        print(f"flag {flag} @ {p:#x}: " + " ".join(f"{x:.3f}" for x in ts), flush=True)


if __name__ == "__main__":
    main()
