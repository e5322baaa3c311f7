#!/bin/bash
# Round 3, call I: the tick's tail queue (MRAFT_TICK_STEAL: each XCD's last
# groups claimed dynamically, across XCDs) A/B on the same state copies, at
# 32,768 and 65,536 groups.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3i
mkdir -p "$OUT"
for g in 32768 65536; do
  TICK_GROUPS=$g COPIES=8 REPS=2 VARIANTS="tbase,st512,st256,st128" timeout -k 10 400 python3 -u tools/ab_variants.py \
    > "$OUT/ab_steal_g$g.txt" 2>&1 || { echo "FAILED $g"; tail -5 "$OUT/ab_steal_g$g.txt"; exit 1; }
  echo "== $g"; grep -v "^per copy" "$OUT/ab_steal_g$g.txt" | grep -v amdgpu.ids
done
