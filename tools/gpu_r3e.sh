#!/bin/bash
# Round 3, call E: the ramp at 32,768 groups per GPU (config #4's N = 8 shard):
# dispatch-order experiments (same work, another order) and the per-group
# phase trace (diagnostic build).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3e
mkdir -p "$OUT"
B="python3 -u bench.py --global-groups 32768 --steps 30 --warmup 3 --no-cpu-baseline --no-secondary"
for r in 1 2; do
  for o in natural lpt-xcd taillight0.12 taillight0.25; do
    timeout -k 10 180 $B --group-order $o > "$OUT/$o.$r.json" 2> "$OUT/$o.$r.err" || { echo "FAILED $o"; tail -5 "$OUT/$o.$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/$o.$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$o', $r, round(r['kernel_ms_mean'],4), round(r['kernel_ms_min'],4), round(r['frac'],3))"
  done
done
TRACE_G=32768 TRACE_SAVE=$OUT/trace_g32768.npy MRAFT_LIB=$PWD/tools/variants/libmraft_hip_trace.so \
  timeout -k 10 180 python3 -u tools/trace_tick.py > "$OUT/trace_g32768.txt" 2>&1 || { echo "FAILED trace"; tail -5 "$OUT/trace_g32768.txt"; exit 1; }
head -12 "$OUT/trace_g32768.txt"
