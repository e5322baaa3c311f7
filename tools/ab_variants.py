"""A/B timing of tick-kernel variants on the SAME state copies (GPU box).

Every tools/variants/libmraft_hip_<tag>.so (tools/build_variants.sh) is loaded
into this one process (RTLD_LOCAL, one engine each) and the tick is timed per
copy, variants interleaved, so the placement lottery of the 5 GiB log image
(some copies are ~12 % slower, whichever kernel runs) is the
same for every variant. Each variant's result on copy 0 is checked against the
first variant's (group flags and state checksums)."""
import ctypes
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from multiraft_amd import DEVICE, synth_seed, synth_tick_state
    from multiraft_amd._abi import MraftSoa, STATE_FIELDS, soa_of
    G = int(os.environ.get("TICK_GROUPS", 65536))  # (bash reserves GROUPS)
    P, L = 5, 4096
    N = int(os.environ.get("COPIES", 8))
    R = int(os.environ.get("REPS", 2))
    # VARIANTS: comma-separated tags or globs (the first one is the reference)
    libs = []
    for pat in os.environ.get("VARIANTS", "*").split(","):
        libs += sorted(glob.glob(os.path.join(ROOT, "tools", "variants", f"libmraft_hip_{pat}.so")))
    tags = [os.path.basename(p)[len("libmraft_hip_"):-3] for p in libs]
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    del st
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(N)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    engines = []
    for p in libs:
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        lib.mraft_create.argtypes = [ctypes.c_int32] * 4 + [ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
        lib.mraft_bind_state.argtypes = [ctypes.c_void_p, ctypes.POINTER(MraftSoa)]
        lib.mraft_set_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.mraft_replicate_tick.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        h = ctypes.c_void_p()
        assert lib.mraft_create(G, P, L, 0, 1, ctypes.byref(h)) == 0
        assert lib.mraft_set_stream(h, stream.cuda_stream) == 0
        engines.append((lib, h))
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    times = np.zeros((len(libs), N, R))
    ref = None
    for r in range(R):
        for i, c in enumerate(clones):
            for vi, (lib, h) in enumerate(engines):
                for k in c:
                    c[k].copy_(master[k])
                soa = soa_of(c)
                assert lib.mraft_bind_state(h, ctypes.byref(soa)) == 0
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                assert lib.mraft_replicate_tick(h, lp_d.data_ptr(), gf.data_ptr(), DEVICE) == 0
                b.record(stream)
                torch.cuda.synchronize()
                times[vi, i, r] = a.elapsed_time(b)
                if r == 0 and i == 0:
                    sig = [int(gf.sum())] + [int((c[k].to(torch.int64) * (1 + torch.arange(c[k].numel(), device=dev) % 7)).sum())
                                             for k in STATE_FIELDS if k != "log_term"]
                    live = c["log_term"].view(G * P, L)
                    w = 1 + torch.arange(G * P, device=dev, dtype=torch.int64) % 13
                    sig.append(int((live.sum(dim=1, dtype=torch.int64) * w).sum()))
                    sig.append(int((live[:, 1::7].sum(dim=1, dtype=torch.int64) * w).sum()))
                    if ref is None:
                        ref = sig
                    elif sig != ref:
                        print(f"MISMATCH {tags[vi]} vs {tags[0]}", flush=True)
    per_copy = times.min(axis=2)  # [variant, copy]
    base = per_copy[0]
    slow = base > np.median(base) * 1.05
    out = {}
    for vi, t in enumerate(tags):
        out[t] = {"mean_ms": round(float(times[vi].mean()), 4),
                  "copy_min_mean_ms": round(float(per_copy[vi].mean()), 4),
                  "fast_copies_ms": round(float(per_copy[vi][~slow].mean()), 4) if (~slow).any() else None,
                  "slow_copies_ms": round(float(per_copy[vi][slow].mean()), 4) if slow.any() else None}
        print(t, json.dumps(out[t]), flush=True)
    print("per copy:", json.dumps({t: [round(x, 3) for x in per_copy[vi]] for vi, t in enumerate(tags)}))


if __name__ == "__main__":
    main()
