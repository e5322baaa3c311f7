"""Per-kernel HBM bytes of the message path (tools/gpu_r5.sh pmcmsg: FETCH_SIZE
and WRITE_SIZE passes over tools/ab_message_path.py), calibrated with the
factors of profiles/pmc_traffic_s2.json. Per kernel: dispatches, and the
average read / written MB per dispatch over its dispatches of the largest
grid size (the one-pipeline steps' full-batch launches; fixed-grid kernels
average over every dispatch).

Usage: python tools/pmc_msg.py <fetch_dir> <write_dir> [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ref = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_s2.json")))


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][-50:]


def per_kernel(d, counter):
    v = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                v[short(r["Kernel_Name"])].append((int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))
    out = {}
    for k, xs in v.items():
        grids = [g for g, _ in xs]
        sel = [x for g, x in xs if g == max(grids)]
        out[k] = {"dispatches": len(xs), "grid_max": max(grids), "avg_at_grid_max": sum(sel) / len(sel)}
    return out


fe, wr = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
res = {}
for k in sorted(set(fe) | set(wr)):
    if not k.startswith("k_"):
        continue
    r = fe.get(k, {}).get("avg_at_grid_max", 0) * 1024 * ref["fetch_factor"] / 1e6
    w = wr.get(k, {}).get("avg_at_grid_max", 0) * 1024 * ref["write_factor"] / 1e6
    res[k] = {"dispatches": fe.get(k, wr.get(k, {})).get("dispatches"), "read_MB": round(r, 2), "write_MB": round(w, 2)}
print(json.dumps(res, indent=1))
if len(sys.argv) > 3:
    json.dump(res, open(sys.argv[3], "w"), indent=1)
