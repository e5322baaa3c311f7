#!/bin/bash
# Round 3, call AC: CU reservation for the overlapped fan-in at config #4's
# 32,768-group shard (one-rank RCCL communicator, --fanin-at-1): 0, 1, 2, 4
# and 8 reserved CUs, two interleaved passes, tick and gather times per run.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ac
mkdir -p "$OUT"
for rep in 1 2; do
  for c in 8 0 1 2 4; do
    timeout -k 10 300 python3 -u bench.py --fanin-at-1 --global-groups 32768 --fanin-cus $c --no-secondary \
      --no-cpu-baseline > "$OUT/cus$c.$rep.json" 2> "$OUT/cus$c.$rep.err" || { echo "FAILED cus=$c"; tail -5 "$OUT/cus$c.$rep.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/cus$c.$rep.json')); r=d['roofline']
c=d['config']; print('cus=$c rep=$rep', round(d['ms_per_step'],4), round(r['kernel_ms_mean'],4), round(r['frac'],3), 'ag', round(c['allgather_ms_mean'],4), 'gap', round(c['step_minus_kernel_ms'],4))"
  done
done
echo done
