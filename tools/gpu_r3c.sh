#!/bin/bash
# Round 3, call C: the many-group scenario replays on the GPU, then the whole
# -m gpu suite.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3c
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=500
timeout -k 10 1000 python3 -u -m pytest tests/test_sim_many.py -m gpu -x -v -s --timeout 900 --timeout-method thread \
  > "$OUT/many.txt" 2>&1 || { echo "FAILED many rc=$?"; tail -30 "$OUT/many.txt"; exit 1; }
grep -E "groups x|passed|failed" "$OUT/many.txt" | tail -12
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_sim_many.py > "$OUT/gpu_tests.txt" 2>&1 || { echo "FAILED suite rc=$?"; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -3 "$OUT/gpu_tests.txt"
