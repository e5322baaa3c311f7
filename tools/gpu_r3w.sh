#!/bin/bash
# Round 3, call W: persist marks at the end of the tick's and the handler's
# waves as non-returning atomic ORs (no dependent load at the end of every
# wave) — the whole -m gpu suite, tick A/B against HEAD on the same state
# copies at 32,768 and 65,536 groups, message path A/B.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3w
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=500
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "FAILED suite rc=$?"; grep -E "FAILED|Error" "$OUT/gpu_tests.txt" | head; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
for g in 32768 65536; do
  TICK_GROUPS=$g COPIES=8 REPS=3 VARIANTS="head,new" timeout -k 10 500 python3 -u tools/ab_variants.py \
    > "$OUT/ab_pdirty_g$g.txt" 2>&1 || { echo "FAILED $g"; tail -5 "$OUT/ab_pdirty_g$g.txt"; exit 1; }
  echo "== $g"; grep -v "^per copy" "$OUT/ab_pdirty_g$g.txt" | grep -v amdgpu.ids
done
REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
