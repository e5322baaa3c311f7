#!/bin/bash
# Round 3, call AD: wave priority in the tick (MRAFT_TICK_PRIO: 1 = header at
# s_setprio 3 and the pass at 0, 2 = the pass at 2 and the rest at 0) against
# the default, on the same state copies, at 32,768 and 65,536 groups.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ad
mkdir -p "$OUT"
for g in 32768 65536; do
  TICK_GROUPS=$g COPIES=8 REPS=3 VARIANTS="base,prio1,prio2" timeout -k 10 500 python3 -u tools/ab_variants.py \
    > "$OUT/ab_prio_g$g.txt" 2>&1 || { echo "FAILED $g"; tail -5 "$OUT/ab_prio_g$g.txt"; exit 1; }
  echo "== $g"; grep -v "^per copy" "$OUT/ab_prio_g$g.txt" | grep -v amdgpu.ids
done
echo done
