"""Writes profiles/config4_n1_anchor.json (read by bench.py's N > 1 lines as
strong_scaling_reference_ms, matched by tick shards per GPU) from a one-GPU
bench.py result line that carries secondary.config4_one_gpu.

Usage: python tools/write_anchor.py <bench_output.json> <tag>
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4 = d["secondary"]["config4_one_gpu"]
out = {"tag": sys.argv[2], "groups": c4["groups"], "steps": c4["steps"], "by_shards": {}}
for sk, c in c4["by_shards"].items():
    r = c["roofline"]
    out["by_shards"][sk] = {"ms_per_step": c["ms_per_step"], "kernel_ms_mean": r["kernel_ms_mean"],
                            "decisions_per_s": c["decisions_per_s"], "frac": r["frac"],
                            "algorithmic_bytes": r["algorithmic_bytes"]}
json.dump(out, open(os.path.join(ROOT, "profiles", "config4_n1_anchor.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
