"""Diagnostic: which source did the differing words of the ring2 case come from?"""
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
for trial in range(3):
    for cap in (None, 0):
        rng = np.random.default_rng(18)
        st, lp, _ = synth_tick_state(G, P, L, seed=78)
        st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(0, G, 3), 2)
        pr = logical_logs(st, G, P, L)
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
        live = w["last_index"] - w["dummy_index"]
        bad = [r for r in range(G * P) if not np.array_equal(lg[r, :live[r] + 1], lw[r, :live[r] + 1])]
        print(f"trial {trial} cap {cap}: rep eq {np.array_equal(rep, orep)} err eq {np.array_equal(herr, oherr)} "
              f"bad rows {bad[:12]} ({len(bad)})")
        for r in bad[:4]:
            j = np.nonzero(batch["slot"] == r)[0][0]
            a = batch[j]
            src = int(a["entries_offset"]) // L
            off = int(a["entries_offset"]) % L
            diff = np.nonzero(lg[r, :live[r] + 1] != lw[r, :live[r] + 1])[0]
            # Index i of the message's entries = prev + 1 + k, at source logical position off + k
            ks = diff - (int(a["prev_log_index"]) + 1)
            print(f"   row {r} <- src {src} prev {int(a['prev_log_index'])} n {int(a['n_entries'])}: diff idx {diff[:6]} "
                  f"gpu {lg[r, diff[:6]]} oracle {lw[r, diff[:6]]} src pristine {pr[src, off + ks[:6]]} "
                  f"src final gpu {lg[src, off + ks[:6]]} follower pristine {pr[r, diff[:6]]}")
