#!/bin/bash
# Round 3, call P: the AppendEntries handler without scratch spills (LDS
# stash through plain LDS accesses, kernel arguments re-read after the pass)
# — parity of the message path, A/B against HEAD on the config #3 message
# path, and per-kernel HBM traffic of the message path.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3p
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  STEPS=4 timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o p -- python3 tools/bench_items.py > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.err; exit 1; }
done
echo done
