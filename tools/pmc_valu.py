"""VALU issue of the config #5 election storm (k_election_rounds<7>) from a
rocprofv3 --pmc pass of bench_election.py (tools/gpu_r5.sh step `valu`) into
profiles/pmc_valu_config5.json, read by bench.py / bench_election.py as the
storm's roofline (bound: VALU issue).

Model (MI355X_MICROARCH.md, Execution model): 4 SIMD-32 per CU, 256 CUs; a
wave64 VALU instruction occupies its SIMD's vector issue for 2 cycles when
enough waves are resident, so the chip issues at most 1,024 / 2 wave
instructions per cycle. frac = SQ_INSTS_VALU x 2 / (1,024 x clock x kernel
time), at the 2.4 GHz peak engine clock (a lower clock only raises it).
SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) gives the busy view
beside it: 4 x SQ_ACTIVE_INST_VALU / (1,024 SIMDs x GRBM_GUI_ACTIVE).

Usage: python tools/pmc_valu.py <tag> <counter dir> [bench json]
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_election_rounds<7>"


def elect_src_sha() -> str:
    h = hashlib.sha1()
    for f in ("mraft_elect.hip", "mraft_device.h"):
        h.update(open(os.path.join(ROOT, "multiraft_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:12]


def main():
    tag, d = sys.argv[1], sys.argv[2]
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"tag": tag, "kernel": KERNEL, "kernel_src_sha": elect_src_sha(), "counters_per_launch": avg,
           "dispatches": max((len(v) for v in vals.values()), default=0),
           "model": "wave64 VALU instruction = 2 issue cycles of one SIMD-32; 1,024 SIMDs; 2.4 GHz",
           "simds": 1024, "clock_hz": 2.4e9, "cycles_per_valu_inst": 2}
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        b = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
        km = b.get("kernel_ms_mean") or b.get("roofline", {}).get("kernel_ms_mean")
        if km and "SQ_INSTS_VALU" in avg:
            out["kernel_ms_mean_same_run"] = km
            out["frac_same_run"] = avg["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * km / 1e3)
    if avg.get("GRBM_GUI_ACTIVE") and out.get("kernel_ms_mean_same_run"):
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: the engine clock the
        # launch actually ran at, and the fraction at that clock
        clk = avg["GRBM_GUI_ACTIVE"] / 8 / (out["kernel_ms_mean_same_run"] / 1e3)
        out["clock_hz_measured"] = clk
        out["frac_at_measured_clock"] = avg["SQ_INSTS_VALU"] * 2 / (1024 * clk * out["kernel_ms_mean_same_run"] / 1e3)
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_valu_config5.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
