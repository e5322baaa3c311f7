"""The fused tick and the message handler on the SAME config #3 state copies,
in one process (where does the tick's 8 % streaming gap to
the handler come from?). Each rep restores one device copy from the pristine
image, runs mraft_replicate_tick on it (one launch, k_tick_group<5,false>),
restores it again and runs gather -> mraft_handle_append_entries_ex by
reference on it (k_ae_set_plan, k_handle_set<4>): both kernels stream the
same merges over the same physical pages. Under `rocprofv3 --pmc` every
dispatch's counters land in the CSV; tools/pmc_kernels.py averages them per
kernel. Prints one JSON line with the HIP-event times of both.

Env: REPS (default 4), COPY (which of COPIES resident copies to use for the
reps, default 0: one copy, so placement is the same for both kernels)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from multiraft_amd import DEVICE, Engine, _abi, synth_seed, synth_tick_state
    G, P, L = 65536, 5, 4096
    reps = int(os.environ.get("REPS", 4))
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    copy = {k: v.clone() for k, v in master.items()}
    lib = _abi.lib()
    ldr = (np.arange(G) * P + lp).repeat(P - 1)
    q = np.tile(np.arange(P - 1), G)
    peers = np.where(q < np.repeat(lp, P - 1), q, q + 1)
    keep = np.repeat(lp >= 0, P - 1)
    slots_d = torch.from_numpy(ldr[keep].astype(np.int32)).to(dev)
    peers_d = torch.from_numpy(peers[keep].astype(np.int32)).to(dev)
    n = len(slots_d)
    z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    args, gerr, herr, rep, res = z(n, 10), z(n), z(n), z(n, 4), z(n, 8)
    lp_d = torch.from_numpy(lp).to(dev)
    gf = z(G)
    e = Engine(G, P, L, device=0, alloc=False)
    st_ = torch.cuda.ExternalStream(e.stream(), device=dev)
    out = {"tick_ms": [], "handle_ms": [], "gather_ms": []}

    def restore():
        with torch.cuda.stream(st_):
            for k, v in master.items():
                copy[k].copy_(v)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    for r in range(reps + 1):
        restore()
        e.bind(copy)
        a, b = ev(), ev()
        a.record(st_)
        e.replicate_tick(lp_d, gf, where=DEVICE)
        b.record(st_)
        restore()
        e.bind(copy)
        c, d, f = ev(), ev(), ev()
        c.record(st_)
        assert lib.mraft_gather_append_args(e._h, slots_d.data_ptr(), peers_d.data_ptr(), n, args.data_ptr(),
                                            gerr.data_ptr(), DEVICE) == 0, _abi.last_error()
        d.record(st_)
        assert lib.mraft_handle_append_entries_ex(e._h, args.data_ptr(), n, None, 0, rep.data_ptr(), res.data_ptr(),
                                                  herr.data_ptr(), DEVICE) == 0, _abi.last_error()
        f.record(st_)
        e.synchronize()
        if r:  # rep 0 warms up
            out["tick_ms"].append(a.elapsed_time(b))
            out["gather_ms"].append(c.elapsed_time(d))
            out["handle_ms"].append(d.elapsed_time(f))
    assert int(gerr.abs().sum()) == 0 and int(herr.abs().sum()) == 0
    e.close()
    print(json.dumps({k: [round(x, 4) for x in v] for k, v in out.items()}))


if __name__ == "__main__":
    main()
