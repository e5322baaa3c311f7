"""Instruction account of a kernel's loops: compiles a
source for gfx950 to device assembly in a temporary directory, cuts out one
kernel and counts its instructions per loop depth and per basic block, by
class (VALU, SALU, LDS, SMEM, VMEM, control), from the compiler's own loop
annotations ("Loop Header: Depth=N", "in Loop: Header=... Depth=N").

  python3 tools/isa_account.py SRC KERNEL_SUBSTR [--define X=Y ...] [--json OUT]

Used on k_election_rounds<7> (mraft_elect.hip): the per-candidate delivery
loop (depth 2) and the per-round body (depth 1). CPU only."""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import tempfile

CONTROL = ("s_branch", "s_cbranch", "s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_setprio", "s_sleep")


def classify(mn: str) -> str:
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if mn.startswith(CONTROL):
        return "control"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def compile_asm(src: str, defines: list[str], out_dir: str) -> str:
    asm = os.path.join(out_dir, "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-mcode-object-version=5",
           "-munsafe-fp-atomics", "--cuda-device-only", "-S", src, "-o", asm] + ["-D" + d for d in defines]
    subprocess.run(cmd, check=True, capture_output=True)
    return asm


def kernel_body(asm: str, substr: str) -> list[str]:
    lines = open(asm).read().splitlines()
    start = next(i for i, l in enumerate(lines)
                 if re.match(r"^[A-Za-z_]\S*:", l) and substr in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def account(body: list[str]) -> dict:
    blocks, cur, depth = [], None, 0
    for l in body:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?\s*(;.*)?$", l)
        if m:
            note = m.group(2) or ""
            d = re.search(r"Depth=(\d+)", note)
            depth = int(d.group(1)) if d else 0
            cur = {"block": m.group(1).lstrip("; "), "depth": depth, "counts": {}}
            blocks.append(cur)
            continue
        t = l.strip()
        if cur is not None and t.startswith(";") and not cur["counts"]:
            # the label's continuation comments ("=>  This Inner Loop Header: Depth=2")
            d = re.search(r"Depth=(\d+)", t)
            if d:
                cur["depth"] = max(cur["depth"], int(d.group(1)))
            continue
        if not t or t.startswith((";", ".")) or cur is None:
            continue
        mn = t.split()[0]
        c = classify(mn)
        cur["counts"][c] = cur["counts"].get(c, 0) + 1
    per_depth: dict[int, dict] = {}
    for b in blocks:
        agg = per_depth.setdefault(b["depth"], {})
        for k, v in b["counts"].items():
            agg[k] = agg.get(k, 0) + v
    return {"blocks": blocks, "per_depth": {str(k): v for k, v in sorted(per_depth.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel")
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        body = kernel_body(compile_asm(a.src, a.define, td), a.kernel)
    r = account(body)
    r.update({"src": a.src, "kernel": a.kernel, "defines": a.define, "instructions": sum(
        sum(b["counts"].values()) for b in r["blocks"])})
    for d, c in r["per_depth"].items():
        print(f"depth {d}: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    if a.json:
        json.dump(r, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
