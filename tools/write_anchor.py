"""Writes profiles/config4_n1_anchor.json (read by bench.py's N > 1 lines as
strong_scaling_reference_ms) from a one-GPU bench.py result line that carries
secondary.config4_one_gpu.

Usage: python tools/write_anchor.py <bench_output.json> <tag>
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4 = d["secondary"]["config4_one_gpu"]
out = {"tag": sys.argv[2], "groups": c4["groups"], "steps": c4["steps"], "ms_per_step": c4["ms_per_step"],
       "kernel_ms_mean": c4["roofline"]["kernel_ms_mean"], "decisions_per_s": c4["decisions_per_s"],
       "frac": c4["roofline"]["frac"], "algorithmic_bytes": c4["roofline"]["algorithmic_bytes"]}
json.dump(out, open(os.path.join(ROOT, "profiles", "config4_n1_anchor.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
