"""Summarises tools/exp_pmc.sh: per variant, tick kernel time and the
FETCH_SIZE / WRITE_SIZE of the tick kernel (x1024 B; FETCH_SIZE x2 for the
gfx950 wide-read under-count, MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for j in sorted(glob.glob(os.path.join(d, "*.json"))):
    tag = os.path.basename(j)[:-5]
    b = json.load(open(j))
    r = b["roofline"]
    row = [tag, f"{r['kernel_ms_mean'] * 1e3:.1f}us", f"frac={r['frac']:.3f}",
           f"algo={r['algorithmic_bytes_per_launch'] / 1e6:.1f}MB"]
    for c in sorted(glob.glob(os.path.join(d, f"{tag}_*"))):
        if not os.path.isdir(c):
            continue
        cname = os.path.basename(c)[len(tag) + 1:]
        vals = {}
        for f in glob.glob(os.path.join(c, "**", "*counter_collection.csv"), recursive=True):
            for rr in csv.DictReader(open(f)):
                if "k_tick_group<5, false>" in rr["Kernel_Name"]:
                    vals.setdefault(rr["Counter_Name"], []).append(float(rr["Counter_Value"]))
        for k, v in sorted(vals.items()):
            x = sum(v) / len(v)
            if k in ("FETCH_SIZE", "WRITE_SIZE"):
                x = x * 1024 * (2 if k == "FETCH_SIZE" else 1) / 1e6
                row.append(f"{k}={x:.1f}MB")
            else:
                row.append(f"{k}={x:.4g}")
    print("  ".join(row))
