#!/bin/bash
# Round 3, call Z: rocprofv3 kernel trace + stats of the default bench line on
# the final round-3 tree (the tick kernel's mean under the profiler beside the
# line's own HIP-event mean), then the default bench line again unprofiled.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3z
mkdir -p "$OUT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py \
  > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || { echo "FAILED kt"; tail -5 "$OUT/kt_bench.err"; exit 1; }
cp "$(find "$OUT/kt" -name 'kt_kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
grep -E "k_tick_group|k_handle_set|k_fold|k_election" "$OUT/kernel_stats.csv" | cut -c1-160
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED bench"; tail -5 "$OUT/bench.err"; exit 1; }
tail -3 "$OUT/bench.err"
echo done
