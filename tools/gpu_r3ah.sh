#!/bin/bash
# Round 3, call AH: the final tree's default bench line again on another box,
# and the 32,768-group shard (config #4's per-GPU size at N = 8) with the
# one-rank RCCL fan-in, shards 2 (default) and 1.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_v16
mkdir -p "$OUT"
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED bench"; tail -5 "$OUT/bench.err"; exit 1; }
for sh in 2 1; do
  timeout -k 10 300 python3 -u bench.py --shards $sh --fanin-at-1 --global-groups 32768 --no-secondary --no-cpu-baseline > "$OUT/g32768_fanin_s$sh.json" 2> "$OUT/g32768_fanin_s$sh.err" || { echo "FAILED g32k s$sh"; tail -5 "$OUT/g32768_fanin_s$sh.err"; exit 1; }
done
for f in bench g32768_fanin_s2 g32768_fanin_s1; do python3 -c "
import json; d=json.load(open('$OUT/$f.json')); r=d['roofline']; c=d['config']
print('$f', round(d['ms_per_step'],4), round(r['kernel_ms_mean'],4), round(r['frac'],3), c.get('shards_per_gpu'), c.get('allgather_ms_mean'), round(c['step_minus_kernel_ms'],4), (r.get('placement_probe') or {}).get('populations'))"; done
echo done
