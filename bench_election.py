"""Secondary benchmark, SURVEY.md §8d config #5 (election storm): 65,536
groups x 7 peers, R = 64 election rounds per launch (timeouts ->
StartElection, every RequestVote, every tally; mraft_election_rounds).
One step = one launch over a fresh HBM-resident copy of the seeded state.
Prints one JSON line. The headline benchmark is bench.py (config #3)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--peers", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import torch

    from multiraft_amd import DEVICE, Engine, synth_election_state, synth_seed
    G, P, R, L, K, W = a.groups, a.peers, a.rounds, 8, a.steps, a.warmup
    dev = torch.device("cuda", 0)
    st, mask = synth_election_state(G, P, L, seed=synth_seed(5), rounds=R)
    nc = np.unpackbits(mask[..., None], axis=-1).sum(axis=-1)  # timed-out peers per (round, group)
    rv_upper = int(nc.sum()) * (P - 1)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    mask_d = torch.from_numpy(mask).to(dev)
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(K + 1)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = Engine(G, P, L, alloc=False)
    eng.set_stream(stream.cuda_stream)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for i in range(W):
        eng.bind(clones[K])
        eng.election_rounds(mask_d, gf, where=DEVICE)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        eng.bind(clones[i])
        ev[i][0].record(stream)
        eng.election_rounds(mask_d, gf, where=DEVICE)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ker = float(np.mean([x.elapsed_time(y) for x, y in ev])) / 1e3
    # words touched per launch: 6 scalars + last term per replica read, 4 written,
    # the round masks, and matchIndex/nextIndex rows of elected replicas.
    from bench import valu_roofline  # the VALU-issue roofline from the committed PMC pass
    flags = gf.cpu().numpy()
    bytes_launch = G * P * (7 + 4) * 4 + mask.size + int(((flags & 128) != 0).sum()) * P * 2 * 4
    out = {"metric": "election-storm rounds/sec @64k groups×7 peers (R=64 per launch)",
           "value": G * R * K / dt, "unit": "group-rounds/s", "n_gpus": 1, "steps": K, "warmup": W,
           "ms_per_step": dt / K * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "int32",
           "data": "synthetic: seeded config-#5 generator (mraft_synth_election_state)",
           "config": {"workload": "config #5 election storm", "groups": G, "peers": P, "rounds": R,
                      "requestvotes_per_launch_upper_bound": rv_upper,
                      "groups_with_new_leader": int(((flags & 128) != 0).sum())},
           "roofline": {"bound": "valu", "achieved": bytes_launch / ker / 1e9, "peak": 8000.0,
                        "unit": "GB/s", "frac": bytes_launch / ker / 8e12, "traffic": None,
                        "kernel": f"k_election_rounds<{P}>", "kernel_ms_mean": ker * 1e3,
                        "note": ("VALU/issue-bound, not HBM: every replica's election state stays in "
                                 "registers for all R rounds (HBM touched once in, once out); the GB/s "
                                 "here are only the state bytes per launch")},
           "requestvotes_per_sec": rv_upper * K / dt,
           "valu_roofline": valu_roofline(ker * 1e3),
           "cpu_baseline": None}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle_lib import Oracle  # checker / CPU baseline only
        Gs = 8192
        from bench import cpu_share  # affinity, capped by the cgroup quota
        share = cpu_share()
        threads = share["threads"]
        sst, smask = synth_election_state(G, P, L, seed=synth_seed(5), rounds=R, g_begin=0, g_end=Gs)
        o = Oracle(Gs, P, L, sst)

        def run(nt, budget):
            done, spent = 0, 0.0
            while spent < budget:
                for k, v in sst.items():  # pristine state, untimed
                    np.copyto(o.st[k], v)
                t = time.perf_counter()
                o.election_rounds(smask, nthreads=nt)
                spent += time.perf_counter() - t
                done += Gs * R
            return done / spent, spent

        v1, _ = run(1, min(2.0, a.cpu_seconds / 4))
        vt, spent = run(threads, a.cpu_seconds)
        out["cpu_baseline"] = {"value": vt, "unit": "group-rounds/s", "cores": threads,
                               "kind": "port", "single_thread_value": v1, "nproc": os.cpu_count(),
                               "cores_source": f"sched_getaffinity {share['affinity']}, cgroup quota "
                                               f"{share['cgroup_quota']}",
                               "sample": f"oracle ora_election_rounds on groups 0..{Gs - 1}, {R} rounds, "
                                         f"fresh state per pass, {spent:.1f} s on {threads} threads; "
                                         f"1 thread: {v1:.4g} group-rounds/s"}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
