#!/bin/bash
# Round 3, call R: (1) tick A/B — the launch's last N workgroups stream their
# copy-only loop D chunks ahead (MRAFT_TICK_TAIL_N / _D), same state copies for
# every variant, at 32,768 and 65,536 groups; (2) k_fold_scan knobs (replies
# per wave, terms per round trip) on the config #3 message path, with a
# kernel trace of the default library's message path.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3r
mkdir -p "$OUT"
for g in 32768 65536; do
  TICK_GROUPS=$g COPIES=8 REPS=2 VARIANTS="tbase,t2k_d2,t4k_d2,t8k_d2,t4k_d3,t8k_d3" timeout -k 10 500 python3 -u tools/ab_variants.py \
    > "$OUT/ab_tail_g$g.txt" 2>&1 || { echo "FAILED $g"; tail -5 "$OUT/ab_tail_g$g.txt"; exit 1; }
  echo "== $g"; grep -v "^per copy" "$OUT/ab_tail_g$g.txt" | grep -v amdgpu.ids
done
PROFILE=1 REPS=2 VARIANTS="f*" bash tools/tune_items.sh || exit 1
