#!/bin/bash
# Round 3, call X: the record run on the current sources — smoke(), the whole
# -m gpu suite (many-group replays included), the default bench line, and the
# message path's kernel trace and per-kernel HBM traffic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3x
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "FAILED smoke"; tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
export MRAFT_SIM_PROGRESS=500
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "FAILED suite rc=$?"; grep -E "FAILED|Error" "$OUT/gpu_tests.txt" | head; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
tail -4 "$OUT/bench.err"
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o items -- python3 tools/bench_items.py > "$OUT/items_kt.json" 2> "$OUT/items_kt.err" || { echo "FAILED trace"; tail -5 "$OUT/items_kt.err"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  STEPS=4 timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o p -- python3 tools/bench_items.py > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.err; exit 1; }
done
echo done
