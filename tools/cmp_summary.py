"""Per-byte comparison of the fused tick and the message handler on the same
state copy (tools/cmp_tick_handler.py under the counter passes of
tools/gpu_r5.sh `cmp`): for k_tick_group<5, false> and k_handle_set<4, 0>,
the calibrated HBM bytes (FETCH_SIZE x 1024 x 2, WRITE_SIZE x 1024, the
gfx950 factors of profiles/pmc_traffic_s2.json), the kernel time (HIP events
of the unprofiled run), and every counter per MB moved and per microsecond,
with the ratio tick / handler. The counter whose per-byte (or per-us) value
differs most is the candidate for the tick's lower streaming rate.

Usage: python tools/cmp_summary.py <gpurun_out/TAG> [out.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TICK, HAND = "k_tick_group<5, false>", "k_handle_set<4, 0>"


def main():
    d = sys.argv[1]
    c = json.load(open(os.path.join(d, "cmp_counters.json")))
    t = json.loads(open(os.path.join(d, "cmp_times.json")).read().strip().splitlines()[-1])
    ref = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_s2.json")))
    ms = {TICK: sum(t["tick_ms"]) / len(t["tick_ms"]), HAND: sum(t["handle_ms"]) / len(t["handle_ms"])}
    out = {"kernels": {}, "ratios": {}}
    for k in (TICK, HAND):
        x = c.get(k, {})
        rd = x.get("FETCH_SIZE", 0) * 1024 * ref["fetch_factor"]
        wr = x.get("WRITE_SIZE", 0) * 1024 * ref["write_factor"]
        mb = (rd + wr) / 1e6
        row = {"read_MB": rd / 1e6, "write_MB": wr / 1e6, "moved_MB": mb, "event_ms": ms[k],
               "physical_TBps": (rd + wr) / (ms[k] / 1e3) / 1e12 if ms[k] else None,
               "per_MB": {n: v / mb for n, v in x.items() if not n.startswith("_") and mb}}
        if x.get("SQ_WAVE_CYCLES"):
            row["wait_any_frac"] = x.get("SQ_WAIT_ANY", 0) / x["SQ_WAVE_CYCLES"]
            row["active_any_frac"] = x.get("SQ_ACTIVE_INST_ANY", 0) / x["SQ_WAVE_CYCLES"]
        if x.get("TCC_HIT") is not None and x.get("TCC_MISS") is not None:
            row["tcc_hit_rate"] = x["TCC_HIT"] / max(1.0, x["TCC_HIT"] + x["TCC_MISS"])
        if x.get("GRBM_GUI_ACTIVE"):
            g = x["GRBM_GUI_ACTIVE"]
            for n in ("TCC_EA0_RDREQ_LEVEL", "TCC_EA0_WRREQ_LEVEL"):
                if n in x:
                    row[n + "_per_cycle"] = x[n] / g
        out["kernels"][k] = row
    a, b = out["kernels"][TICK], out["kernels"][HAND]
    for n in sorted(set(a["per_MB"]) & set(b["per_MB"])):
        if b["per_MB"][n]:
            out["ratios"][n] = a["per_MB"][n] / b["per_MB"][n]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
