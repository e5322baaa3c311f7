#!/bin/bash
# Round 3, call AG: the sharded-tick parity test, then a rocprofv3 kernel
# trace + stats of the default bench line (two shards on dedicated queues).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ag
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "shards or tick_small" --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py --no-cpu-baseline \
  > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || { echo "FAILED kt"; tail -5 "$OUT/kt_bench.err"; exit 1; }
cp "$(find "$OUT/kt" -name 'kt_kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
cp "$(find "$OUT/kt" -name 'kt_kernel_trace.csv' | head -1)" "$OUT/kernel_trace.csv"
grep -E "k_tick_group" "$OUT/kernel_stats.csv" | cut -c1-200
python3 -c "
import json; d=json.load(open('$OUT/kt_bench.json')); r=d['roofline']; print(d['ms_per_step'], r['kernel_ms_mean'], r['frac'], r['launch_ms_mean'])"
echo done
