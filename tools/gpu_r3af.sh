#!/bin/bash
# Round 3, call AF: bench.py with group shards pipelined over streams
# (--shards, default 2) against one launch per step (--shards 1), on the same
# box: config #3 headline, and the 32,768-group shard with the one-rank RCCL
# fan-in; then the default line in full.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3af
mkdir -p "$OUT"
summ() { python3 -c "
import json,sys; d=json.load(open('$1')); r=d['roofline']; c=d['config']
print('$2', round(d['ms_per_step'],4), 'ker', round(r['kernel_ms_mean'],4), 'frac', round(r['frac'],3), 'launch', r.get('launch_ms_mean'), 'S', c.get('shards_per_gpu'), 'ag', c.get('allgather_ms_mean'), 'gap', round(c['step_minus_kernel_ms'],4))"; }
for rep in 1 2; do
  for sh in 1 2; do
    timeout -k 10 300 python3 -u bench.py --shards $sh --no-secondary --no-cpu-baseline > "$OUT/c3_s$sh.$rep.json" 2> "$OUT/c3_s$sh.$rep.err" || { echo "FAILED c3 s$sh"; tail -5 "$OUT/c3_s$sh.$rep.err"; exit 1; }
    summ "$OUT/c3_s$sh.$rep.json" "c3 shards=$sh rep=$rep"
    timeout -k 10 300 python3 -u bench.py --shards $sh --fanin-at-1 --global-groups 32768 --no-secondary --no-cpu-baseline > "$OUT/g32k_fan_s$sh.$rep.json" 2> "$OUT/g32k_fan_s$sh.$rep.err" || { echo "FAILED g32k s$sh"; tail -5 "$OUT/g32k_fan_s$sh.$rep.err"; exit 1; }
    summ "$OUT/g32k_fan_s$sh.$rep.json" "g32768+fanin shards=$sh rep=$rep"
  done
done
timeout -k 10 500 python3 -u bench.py > "$OUT/default.json" 2> "$OUT/default.err" || { echo "FAILED default"; tail -5 "$OUT/default.err"; exit 1; }
summ "$OUT/default.json" "default"
tail -4 "$OUT/default.err"
echo done
