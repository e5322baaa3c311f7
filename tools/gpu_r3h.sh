#!/bin/bash
# Round 3, call H: copy-loop depth A/B (same state copies for every variant,
# tools/ab_variants.py) at 32,768 and 65,536 groups.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3h
mkdir -p "$OUT"
for g in 32768 65536; do
  TICK_GROUPS=$g COPIES=8 REPS=2 VARIANTS="tbase,cd2,cd3,cd4" timeout -k 10 400 python3 -u tools/ab_variants.py \
    > "$OUT/ab_copydepth_g$g.txt" 2>&1 || { echo "FAILED $g"; tail -5 "$OUT/ab_copydepth_g$g.txt"; exit 1; }
  echo "== $g"; grep -v "^per copy" "$OUT/ab_copydepth_g$g.txt" | grep -v amdgpu.ids
done
REPS=2 VARIANTS="g*" bash tools/tune_items.sh || exit 1
