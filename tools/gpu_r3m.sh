#!/bin/bash
# Round 3, call M: the record run on the current sources — smoke(), the whole
# -m gpu suite (many-group replays included), the default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3m
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "FAILED smoke"; tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
export MRAFT_SIM_PROGRESS=500
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "FAILED suite rc=$?"; grep -E "FAILED|Error" "$OUT/gpu_tests.txt" | head; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
tail -4 "$OUT/bench.err"
