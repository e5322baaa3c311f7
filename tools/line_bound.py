"""Line-granular bound of the config #3 tick's HBM traffic:
the oracle's algorithmic word bitmaps (ora_count_*) rounded up to the memory
lines that hold a counted word, at 32, 64 and 128 B, read and write apart,
beside the measured PMC traffic (profiles/pmc_traffic_s2.json). Traffic
above the line bound is re-reads; between the word count and the line
bound it is the granularity of the ring's ragged ranges.

Usage: python tools/line_bound.py [out.json]   (CPU, ~1 min, ~12 GB)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from multiraft_amd import synth_seed, synth_tick_state  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

G, P, L = 65536, 5, 4096
st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=8)
o = Oracle(G, P, L, st)
rw, ww, _, lines = o.replicate_tick_count(lp, line_words=(8, 16, 32))
out = {"workload": "config #3 tick (65,536 groups x 5 peers x 4,096)",
       "algorithmic_read_bytes": 4 * rw, "algorithmic_write_bytes": 4 * ww,
       "lines": {str(4 * lw): {"read_bytes": 4 * lw * r, "write_bytes": 4 * lw * w}
                 for lw, (r, w) in lines.items()}}
pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_s2.json")))
steps = pmc["launches_per_step"]
out["pmc"] = {"tag": pmc["tag"], "read_bytes": pmc["hbm_read_bytes_per_dispatch"] * steps,
              "write_bytes": pmc["hbm_write_bytes_per_dispatch"] * steps}
for k, v in out["lines"].items():
    v["pmc_read_over_lines"] = out["pmc"]["read_bytes"] / v["read_bytes"]
    v["pmc_write_over_lines"] = out["pmc"]["write_bytes"] / v["write_bytes"]
    v["pmc_total_over_lines"] = (out["pmc"]["read_bytes"] + out["pmc"]["write_bytes"]) / (
        v["read_bytes"] + v["write_bytes"])
print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
