"""Device timeline of a rocprofv3 --kernel-trace run of tools/ab_message_path.py
(or any run with torch.cuda._sleep gates): for each gated section (the
kernels after a spin kernel, up to the next one) the span from the first
kernel's start to the last one's end, the time at least one kernel runs
(union), the time two or more overlap, and per kernel name the launches,
summed duration and the time it runs alone. Idle = span - union: the device
waiting on the host (a plan poll, launch latency) or on dependencies.

Usage: python tools/timeline.py <dir with *_kernel_trace.csv> [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    if m:
        return m.group(1)
    if "sleep" in name.lower() or "spin" in name.lower():
        return "spin"
    return name.split("(")[0][-60:]


def sections(rows):
    rows = sorted(rows, key=lambda r: r[1])
    out, cur = [], None
    for r in rows:
        if r[0] == "spin":
            cur = []
            out.append(cur)
        elif cur is not None:
            cur.append(r)
    return out


def analyse(sec):
    ks = [r for r in sec if r[0].startswith("k_")]
    if not ks:
        return None
    t0, t1 = min(r[1] for r in ks), max(r[2] for r in ks)
    ev = sorted([(r[1], 1, r[0]) for r in ks] + [(r[2], -1, r[0]) for r in ks])
    union = multi = 0.0
    alone = defaultdict(float)
    active = defaultdict(int)
    n, last = 0, t0
    for t, d, name in ev:
        dt = t - last
        if n >= 1:
            union += dt
        if n >= 2:
            multi += dt
        if n == 1:
            only = [k for k, v in active.items() if v > 0]
            if only:
                alone[only[0]] += dt
        n += d
        active[name] += d
        last = t
    per = defaultdict(lambda: [0, 0.0])
    for r in ks:
        per[r[0]][0] += 1
        per[r[0]][1] += r[2] - r[1]
    queues = sorted({r[3] for r in ks})
    return {"kernels": len(ks), "queues": len(queues), "span_us": (t1 - t0) / 1e3, "busy_us": union / 1e3,
            "idle_us": (t1 - t0 - union) / 1e3, "overlap_us": multi / 1e3,
            "per_kernel": {k: {"launches": v[0], "sum_us": round(v[1] / 1e3, 1),
                               "alone_us": round(alone[k] / 1e3, 1)} for k, v in sorted(per.items())}}


def main():
    d = sys.argv[1]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q))
    res = [a for a in (analyse(s) for s in sections(rows)) if a]
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
