"""Diagnostic: the ring2 deferred-items case, GPU vs oracle, per stage capacity."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from message_cases import stale_cycle_state  # noqa: E402
from oracle_lib import Oracle, logical_logs  # noqa: E402

from multiraft_amd import Engine, synth_tick_state  # noqa: E402

G, P, L = 256, 5, 128
for cap in (None, 0):
    rng = np.random.default_rng(11 * 1 + len("default"))
    st, lp, _ = synth_tick_state(G, P, L, seed=78)
    st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(0, G, 3), 2)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap is not None:
            e.set_stage_capacity(cap)
        args, gerr = e.gather_append_args(slots, peers)
        batch = args[gerr == 0]
        rep, herr = e.handle_append_entries(batch, None)
        orep, oherr = o.handle_append_entries(batch, None)
        g, w = e.store_state(), o.state()
    lg, lw = logical_logs(g, G, P, L), logical_logs(w, G, P, L)
    print(f"cap {cap}: rep equal {np.array_equal(rep, orep)}, err equal {np.array_equal(herr, oherr)}")
    for k in ("last_index", "commit_index", "current_term", "state", "terms_sorted"):
        d = np.nonzero(g[k] != w[k])[0]
        print(f"  {k} differs at {d[:10]}")
    live = w["last_index"] - w["dummy_index"]
    bad = [r for r in range(G * P) if not np.array_equal(lg[r, :live[r] + 1], lw[r, :live[r] + 1])]
    print("  log rows differing:", bad[:10], len(bad))
    for r in bad[:3]:
        j = np.nonzero(batch["slot"] == r)[0]
        a = batch[j[0]] if len(j) else None
        print("  row", r, "item", a, "rep", rep[j] if len(j) else None, orep[j] if len(j) else None)
        diff = np.nonzero(lg[r, :live[r] + 1] != lw[r, :live[r] + 1])[0]
        print("    first diff at Index", diff[:5], "gpu", lg[r, diff[:8]], "oracle", lw[r, diff[:8]])
        if a is not None:
            src = int(a["entries_offset"]) // L
            print("    source row", src, "pristine entries", st["log_term"][src * L + int(a["entries_offset"]) % L:][:8])
