"""Per-kernel averages of every counter in one or more rocprofv3 --pmc output
directories (each pass its own directory): counters_per_dispatch[kernel]
[counter] = mean over that kernel's dispatches of the largest grid.

Usage: python tools/pmc_kernels.py out.json dir1 [dir2 ...] [--kernels "a;b"]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][-50:]


def collect(dirs, only=None):
    v = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if only and k not in only:
                    continue
                v[k][r["Counter_Name"]].append((int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))
    out = {}
    for k, cs in v.items():
        out[k] = {}
        for c, xs in cs.items():
            gmax = max(g for g, _ in xs)
            sel = [x for g, x in xs if g == gmax]
            out[k][c] = sum(sel) / len(sel)
        out[k]["_dispatches"] = max(len(xs) for xs in cs.values())
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    only = None
    if "--kernels" in args:
        i = args.index("--kernels")
        only = set(args[i + 1].split(";"))
        args = args[:i] + args[i + 2:]
    res = collect(args[1:], only)
    json.dump(res, open(args[0], "w"), indent=1)
    print(json.dumps(res, indent=1))
