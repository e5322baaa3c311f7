"""Summarises a tools/profile_round.sh run (gpurun_out/prof/) into profiles/:

  profiles/<tag>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv           per-kernel FETCH_SIZE / WRITE_SIZE averages
  profiles/pmc_traffic.json        HBM bytes per launch of the tick kernel,
                                   read by bench.py as roofline.traffic

Corrections (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7): counter
KB x 1024; FETCH_SIZE under-reads a streaming read by the factor measured on
tools/calib_pmc (known byte counts, same run), WRITE_SIZE likewise.

Usage: python tools/pmc_summary.py <tag> [prof_dir]
"""
from __future__ import annotations

import csv
import glob
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TICK = "k_tick_group<5, false>"


def kernel_src_sha() -> str:
    h = hashlib.sha1()
    for f in ("mraft_tick.hip", "mraft_tick_body.inc", "mraft_device.h", "mraft_pass.h"):
        h.update(open(os.path.join(ROOT, "multiraft_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:12]


def counter_avgs(path):
    """Per (kernel, counter): the average over the dispatches of the kernel's
    most frequent grid size — the timed steps' launches; a differently sized
    dispatch of the same kernel (the bench's one-launch check after the
    sharded steps) is left out."""
    out = {}
    for f in glob.glob(os.path.join(path, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], r["Counter_Name"])
            out.setdefault(k, []).append((int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))
    avg = {}
    for k, v in out.items():
        grids = [g for g, _ in v]
        mode = max(set(grids), key=grids.count)
        sel = [x for g, x in v if g == mode]
        avg[k] = sum(sel) / len(sel)
    return avg


def main():
    tag = sys.argv[1]
    prof = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = glob.glob(os.path.join(prof, "kt", "*_kernel_stats.csv"))
    if ks:
        shutil.copy(ks[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = counter_avgs(os.path.join(prof, "fetch"))
    write = counter_avgs(os.path.join(prof, "write"))
    calf = counter_avgs(os.path.join(prof, "cal_fetch"))
    calw = counter_avgs(os.path.join(prof, "cal_write"))
    known = json.load(open(os.path.join(prof, "calib.json")))
    # calibration: the dword copy kernel reads and writes known_* bytes
    cf = next(v for (k, c), v in calf.items() if k.startswith("copy_dword(") and c == "FETCH_SIZE")
    cw = next(v for (k, c), v in calw.items() if k.startswith("copy_dword(") and c == "WRITE_SIZE")
    fetch_factor = known["known_read_bytes"] / (cf * 1024)
    write_factor = known["known_write_bytes"] / (cw * 1024)
    rows = []
    for (k, c), v in sorted(fetch.items()):
        w = write.get((k, "WRITE_SIZE"))
        rows.append((k, v, w))
    with open(os.path.join(dst, f"{tag}_pmc.csv"), "w") as f:
        wr = csv.writer(f)
        wr.writerow(["kernel", "FETCH_SIZE_KB_avg", "WRITE_SIZE_KB_avg", "hbm_read_bytes",
                     "hbm_write_bytes"])
        for k, fv, wv in rows:
            wr.writerow([k, fv, wv, fv * 1024 * fetch_factor, (wv or 0) * 1024 * write_factor])
    tick = [(k, fv, wv) for k, fv, wv in rows if TICK in k]
    if not tick:
        print("tick kernel not found in counters")
        return
    k, fv, wv = tick[0]
    bench = {}
    bj = os.path.join(prof, "kt_bench.json")
    if os.path.exists(bj):
        try:
            bench = json.loads(open(bj).read().strip().splitlines()[-1])
        except Exception:
            bench = {}
    cfg = bench.get("config", {})
    S = int(cfg.get("shards_per_gpu", 1) or 1)
    groups = cfg.get("groups_per_gpu", 65536)
    # With S tick shards every step is S launches over G/S groups each (the
    # same kernel): the per-dispatch average times S is one step's traffic.
    out = {
        "tag": tag,
        "kernel": k,
        "kernel_src_sha": kernel_src_sha(),
        "groups": groups,
        "peers": cfg.get("peers", 5),
        "log": cfg.get("log_capacity", 4096),
        "shards": S,
        "launches_per_step": S,
        "fetch_size_kb": fv,
        "write_size_kb": wv,
        "fetch_factor": fetch_factor,
        "write_factor": write_factor,
        "hbm_read_bytes_per_dispatch": fv * 1024 * fetch_factor,
        "hbm_write_bytes_per_dispatch": wv * 1024 * write_factor,
        "hbm_bytes_per_dispatch": fv * 1024 * fetch_factor + wv * 1024 * write_factor,
        "hbm_bytes_per_step": S * (fv * 1024 * fetch_factor + wv * 1024 * write_factor),
        "hbm_bytes_per_launch": S * (fv * 1024 * fetch_factor + wv * 1024 * write_factor),  # per step (older name)
        "algorithmic_bytes_per_launch": bench.get("roofline", {}).get("algorithmic_bytes_per_launch"),
    }
    alg = out["algorithmic_bytes_per_launch"]
    if alg:
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_step"] / alg
    # the headline config keeps the plain name; other group counts (config #4
    # on one GPU) and shard counts get their own file (bench.pmc_json_path)
    name = ("pmc_traffic" + ("" if groups == 65536 else f"_g{groups}") + ("" if S == 1 else f"_s{S}") + ".json")
    json.dump(out, open(os.path.join(dst, name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
