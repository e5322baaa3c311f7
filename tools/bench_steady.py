"""The steady-state measurement of bench.py (secondary.steady_state_config3:
config #3 ticked in place with Start between ticks, full and light tick) alone,
for iterating on the light tick without the whole bench. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from multiraft_amd import synth_seed, synth_tick_state  # noqa: E402


def main():
    G, P, L = 65536, 5, 4096
    dev = torch.device("cuda", 0)
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=16)
    master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
    copies = [{k: v.clone() for k, v in master.items()} for _ in range(3)]
    out = bench.steady_state(master, copies, np.asarray(lp), G, P, L, dev)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
