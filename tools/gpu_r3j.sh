#!/bin/bash
# Round 3, call J: the fold's speculative record load: parity (fold + message
# path tests) and A/B on the config #3 message path.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3j
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_message_path_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/fold_tests.txt" 2>&1 || { echo "FAILED tests"; tail -30 "$OUT/fold_tests.txt"; exit 1; }
tail -2 "$OUT/fold_tests.txt"
REPS=3 VARIANTS="hspec*" bash tools/tune_items.sh || exit 1
