"""Diagnostic: first-mismatch analysis of the rows the deferred path gets wrong."""
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
rng = np.random.default_rng(18)
st, lp, _ = synth_tick_state(G, P, L, seed=78)
st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(0, G, 3), 2)
pr = logical_logs(st, G, P, L)
o = Oracle(G, P, L, st)
with Engine(G, P, L) as e:
    e.load_state(st)
    e.set_stage_capacity(0)
    args, gerr = e.gather_append_args(slots, peers)
    batch = args[gerr == 0]
    rep, herr = e.handle_append_entries(batch, None)
    orep, oherr = o.handle_append_entries(batch, None)
    g, w = e.store_state(), o.state()
lg, lw = logical_logs(g, G, P, L), logical_logs(w, G, P, L)
for r in (345, 619, 976):
    j = np.nonzero(batch["slot"] == r)[0][0]
    a = batch[j]
    src, off = int(a["entries_offset"]) // L, int(a["entries_offset"]) % L
    prev, n = int(a["prev_log_index"]), int(a["n_entries"])
    ent = pr[src, off:off + n]
    fol = pr[r, prev + 1:prev + 1 + n]
    fl = int(st["last_index"][r])
    mm = np.nonzero(ent[:max(0, min(n, fl - prev))] != fol[:max(0, min(n, fl - prev))])[0]
    print(f"row {r}: prev {prev} n {n} fol_last {fl} first mismatch k={mm[:3]} flags {int(a['flags'])} "
          f"head f {int(st['log_head'][r])} src {int(st['log_head'][src])} dummy {int(st['dummy_index'][r])}")
    print("   ent[0:8]", ent[:8], " ent[62:68]", ent[62:68])
    print("   fol[0:8]", fol[:8], " fol[62:68]", fol[62:68])
    print("   gpu[0:8]", lg[r, prev + 1:prev + 9], " gpu[62:68]", lg[r, prev + 63:prev + 69])
    print("   ora[0:8]", lw[r, prev + 1:prev + 9], " ora[62:68]", lw[r, prev + 63:prev + 69])
