"""The config #3 message path alone (bench.message_path: one pipeline with the
per-call split, and two shard pipelines), for A/B runs of library variants
(MRAFT_LIB=tools/variants/libmraft_hip_<tag>.so python tools/ab_message_path.py;
SHARDS=2,3 also times three pipelines).
Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from multiraft_amd import synth_seed, synth_tick_state
    G, P, L = 65536, 5, 4096
    copies_n = int(os.environ.get("COPIES", 13))
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3))
    dev = torch.device("cuda", 0)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    copies = [{k: v.clone() for k, v in master.items()} for _ in range(copies_n)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    one = bench.message_path(master, copies, lp, G, P, L, dev, 1, 8, split=True)
    flat = bench.message_path(master, copies, lp, G, P, L, dev, 1, copies_n - 1)
    out = {"lib": os.environ.get("MRAFT_LIB", "in-tree"), "ms_per_call": one["ms_per_call"],
           "one_pipeline_split_ms": one["device_ms_per_step"], "one_pipeline_ms": flat["device_ms_per_step"]}
    for S in [int(x) for x in os.environ.get("SHARDS", "2").split(",")]:
        r = bench.message_path(master, copies, lp, G, P, L, dev, S, copies_n - 1)
        out["two_pipelines_ms" if S == 2 else f"pipelines_{S}_ms"] = r["device_ms_per_step"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
