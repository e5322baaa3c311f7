"""Per-kernel mean durations and the gaps between consecutive mraft kernels
of the message-level path, from a rocprofv3 kernel trace (csv)."""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mraft" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur, gap = defaultdict(list), defaultdict(list)
prev = None
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("::")[-1]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append((e - s) / 1e3)
    if prev is not None:
        gap[prev[0] + " -> " + name].append((s - prev[1]) / 1e3)
    prev = (name, e)
for k, v in dur.items():
    print(f"{k:40s} n={len(v):3d} mean={sum(v) / len(v):9.2f} us  min={min(v):9.2f}")
for k, v in gap.items():
    if len(v) >= 5:
        v = sorted(v)
        print(f"gap {k:60s} n={len(v):3d} median={v[len(v) // 2]:9.2f} us")
