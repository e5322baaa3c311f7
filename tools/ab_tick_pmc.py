"""Summary of tools/ab_tick_pmc.sh: per library, the tick kernel's HBM bytes
per step (FETCH_SIZE x 1024 x the fetch factor of profiles/pmc_traffic_s2.json,
WRITE_SIZE x 1024 x its write factor, summed over the step's launches) and the
timed lines' kernel time.

Usage: python tools/ab_tick_pmc.py <out_dir> <tag> ..."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import TICK, counter_avgs  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ref = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_s2.json")))
out_dir, tags = sys.argv[1], sys.argv[2:]
res = {}
for t in tags:
    r = {}
    for c, fac in (("FETCH_SIZE", ref["fetch_factor"]), ("WRITE_SIZE", ref["write_factor"])):
        avg = counter_avgs(os.path.join(out_dir, f"pmc_{t}_{c}"))
        v = [x for (k, cn), x in avg.items() if TICK in k and cn == c]
        line = json.loads(open(os.path.join(out_dir, f"pmc_{t}_{c}.json")).read().strip().splitlines()[-1])
        r[c] = v[0] * 1024 * fac * line["roofline"].get("launches_per_step", 1) if v else None
        r["algorithmic_bytes"] = line["roofline"]["algorithmic_bytes_per_launch"]
    lines = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(os.path.join(out_dir, f"{t}.*.json")))]
    r["kernel_ms"] = [round(d["roofline"]["kernel_ms_mean"], 4) for d in lines]
    r["ms_per_step"] = [round(d["ms_per_step"], 4) for d in lines]
    if r["FETCH_SIZE"] and r["WRITE_SIZE"]:
        r["hbm_bytes_per_step"] = r["FETCH_SIZE"] + r["WRITE_SIZE"]
        r["traffic_over_algorithmic"] = r["hbm_bytes_per_step"] / r["algorithmic_bytes"]
    res[t] = r
print(json.dumps(res, indent=1))
