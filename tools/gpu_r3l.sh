#!/bin/bash
# Round 3, call L: the AppendEntries claim check merged into the claim + plan
# (one launch fewer per handle call): parity and A/B on the message path.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3l
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_message_path_gpu.py tests/test_ring.py tests/test_sim2b.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
REPS=3 VARIANTS="j*" bash tools/tune_items.sh || exit 1
