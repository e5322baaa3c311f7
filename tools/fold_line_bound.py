"""Line-granular bound of the reply fold's reads on config #3 (VERDICT r5 item
4; DESIGN.md §5 "Round 6: the fold's bytes"): k_fold reads, per segment (one
leader replica slot s = g * P + leader_peer[g]), the segment bounds and claim
verdict, the claim word at s, seven scalar words at s (term, role, commit,
last, dummy, ring head, terms_sorted), the leader's matchIndex and nextIndex
rows (P words at s * P), its replies' 32-B records, and at most one line of
its log for a1's probe. The SoA arrays are indexed by replica slot and the
leaders are one slot in P, so every one of those word reads touches a line its
neighbours' leaders share only partly. This counts, from config #3's
leader_peer alone, the distinct 64-B and 128-B lines those reads touch — the
bound any kernel reading those words in this layout pays — beside the
algorithmic bytes (tools/msg_words.py fold_words: 16.68 MB per call) and the
measured PMC bytes of k_fold (profiles/r5_v10/message_path_pmc.json).

Usage: python tools/fold_line_bound.py [out.json]   (CPU, seconds)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multiraft_amd import synth_seed, synth_tick_state  # noqa: E402


def lines(byte_lo, byte_hi, line):
    """Distinct lines covering the byte ranges [lo, hi] (each shorter than a line)."""
    return len(np.unique(np.concatenate([byte_lo // line, byte_hi // line])))


def main():
    G, P, L = 65536, 5, 4096
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3), nthreads=8)
    del st
    g = np.flatnonzero(lp >= 0).astype(np.int64)
    s = g * P + lp[g].astype(np.int64)         # leader slots, one segment each
    nseg, nrec = len(s), len(s) * (P - 1)
    out = {"workload": "config #3 reply fold: %d segments, %d records" % (nseg, nrec), "lines": {}}
    for line in (64, 128):
        scal = lines(4 * s, 4 * s + 3, line)                      # one of the seven scalar arrays
        row = lines(4 * s * P, 4 * s * P + 4 * P - 1, line)       # matchIndex or nextIndex row
        claim = lines(8 * s, 8 * s + 7, line)
        rec = -(-32 * nrec // line)
        seg = -(-8 * (nseg + 1) // line) + -(-4 * nseg // line)   # bounds + claim verdicts
        probe_max = nseg                                          # <= one log line per segment
        fixed = (7 * scal + 2 * row + claim + rec + seg) * line
        out["lines"][str(line)] = {
            "scalar_array_bytes": scal * line, "row_array_bytes": row * line, "claim_bytes": claim * line,
            "records_bytes": rec * line, "segments_bytes": seg * line,
            "read_bound_without_probe_bytes": fixed, "read_bound_with_probe_bytes": fixed + probe_max * line}
    pmc = json.load(open(os.path.join(ROOT, "profiles", "r5_v10", "message_path_pmc.json")))["k_fold<5>"]
    out["pmc_k_fold_read_bytes"] = pmc["read_MB"] * 1e6
    out["pmc_k_fold_write_bytes"] = pmc["write_MB"] * 1e6
    out["algorithmic_fold_bytes"] = 16683540
    for k, v in out["lines"].items():
        v["pmc_read_over_bound_lo"] = out["pmc_k_fold_read_bytes"] / v["read_bound_with_probe_bytes"]
        v["pmc_read_over_bound_hi"] = out["pmc_k_fold_read_bytes"] / v["read_bound_without_probe_bytes"]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
