"""Message-level path at config #3 (the entry points a Go host calls for
batches delivered by the network): gather_append_args (a3) ->
handle_append_entries (a4, entries by reference: one wave per set of messages
reading the same leader entries) -> process_append_replies (a2 + a1), all on
device buffers, one fresh HBM-resident state copy per step. Prints per-call
times next to the fused tick's, and the handler's roofline: its algorithmic
words (tools/msg_words.py) over the whole handle call (plan, one host round
trip, kernel: conservative; the kernel alone is in the rocprofv3 summary).
Secondary measurement (the headline is bench.py)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    from multiraft_amd import DEVICE, Engine, synth_seed, synth_tick_state
    from multiraft_amd import _abi
    from msg_words import handle_words
    G, P, L, K = 65536, 5, 4096, int(os.environ.get("STEPS", 10))
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(K + 1)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    lib = _abi.lib()
    ldr = np.repeat(np.arange(G) * P + lp, P - 1).astype(np.int32)
    peers = np.array([p for g in range(G) for p in range(P) if p != lp[g]], np.int32)
    n = len(ldr)
    slots_d, peers_d = torch.from_numpy(ldr).to(dev), torch.from_numpy(peers).to(dev)
    args = torch.zeros((n, 10), dtype=torch.int32, device=dev)   # mraft_ae_args (40 B)
    gerr = torch.zeros(n, dtype=torch.int32, device=dev)
    rep = torch.zeros((n, 4), dtype=torch.int32, device=dev)     # mraft_ae_reply
    herr = torch.zeros(n, dtype=torch.int32, device=dev)
    res = torch.zeros((n, 8), dtype=torch.int32, device=dev)     # mraft_ae_result
    flags = torch.zeros(n, dtype=torch.int32, device=dev)
    ferr = torch.zeros(n, dtype=torch.int32, device=dev)
    seg = torch.arange(0, n + 1, P - 1, dtype=torch.int64, device=dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    names = ("gather", "handle", "assemble", "fold")
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(K)] for k in names + ("tick",)}

    def ck(rc, what):
        assert rc == 0, (what, _abi.last_error())

    def step(i, timed):
        eng.bind(clones[i if timed else K])
        e = ev["gather"][i] if timed else None
        if e: e[0].record(stream)
        ck(lib.mraft_gather_append_args(eng._h, slots_d.data_ptr(), peers_d.data_ptr(), n,
                                        args.data_ptr(), gerr.data_ptr(), DEVICE), "gather")
        if e: e[1].record(stream); ev["handle"][i][0].record(stream)
        ck(lib.mraft_handle_append_entries(eng._h, args.data_ptr(), n, None, 0, rep.data_ptr(),
                                           herr.data_ptr(), DEVICE), "handle")
        if e: ev["handle"][i][1].record(stream); ev["assemble"][i][0].record(stream)
        res[:, 0] = slots_d
        res[:, 1] = peers_d
        res[:, 2] = args[:, 1]
        res[:, 3] = args[:, 3]
        res[:, 4] = args[:, 6]
        res[:, 5:8] = rep[:, 0:3]
        if e: ev["assemble"][i][1].record(stream); ev["fold"][i][0].record(stream)
        ck(lib.mraft_process_append_replies(eng._h, res.data_ptr(), n, seg.data_ptr(), G,
                                            flags.data_ptr(), ferr.data_ptr(), DEVICE), "fold")
        if e: ev["fold"][i][1].record(stream)

    step(0, False)
    torch.cuda.synchronize()
    assert int(gerr.abs().sum()) == 0 and int(herr.abs().sum()) == 0 and int(ferr.abs().sum()) == 0
    hw = handle_words(st, args.cpu().numpy().view(_abi.AE_ARGS).reshape(-1),
                      rep.cpu().numpy().view(_abi.AE_REPLY).reshape(-1), herr.cpu().numpy(), G, P, L)
    t0 = time.perf_counter()
    for i in range(K):
        step(i, True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {k: float(np.mean([a.elapsed_time(b) for a, b in ev[k][:K]])) for k in names}
    # fused tick on fresh copies for comparison
    lp_d = torch.from_numpy(lp).to(dev)
    tk = []
    for i in range(min(K, 5)):
        for k, v in master.items():
            clones[i][k].copy_(v)
        eng.bind(clones[i])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.replicate_tick(lp_d, gf, where=DEVICE)
        b.record(stream)
        torch.cuda.synchronize()
        tk.append(a.elapsed_time(b))
    hb = hw["words"] * 4
    achieved = hb / (out["handle"] * 1e-3)
    print(json.dumps({"config": "#3 message-level path", "items": n,
                      "ms_per_call": {k: round(v, 4) for k, v in out.items()},
                      "ms_per_step_wall": dt / K * 1e3,
                      "decisions_per_s": G * K / dt,
                      "fused_tick_ms": float(np.mean(tk)),
                      "handle": {"sets": hw["sets"], "merges": hw["merges"], "entries_copied": hw["copied"],
                                 "algorithmic_bytes": hb},
                      "roofline": {"kernel": "handle_append_entries (whole call)", "bound": "hbm",
                                   "achieved": round(achieved / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                                   "frac": round(achieved / 8.0e12, 4)}}))


if __name__ == "__main__":
    main()
