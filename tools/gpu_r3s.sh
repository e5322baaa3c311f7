#!/bin/bash
# Round 3, call S: k_fold_scan with one 32-B record per reply (one round trip
# before the scan) and the probe placement (k_fold or k_fold_scan's first
# window) — parity (fold, message path, ring, scenario replays on one group and
# on many), A/B against HEAD on the config #3 message path, kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3s
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=1000
timeout -k 10 900 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py tests/test_ring.py tests/test_sim2b.py tests/test_sim_many.py -m gpu -x -q -s \
  --timeout 800 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
PROFILE=1 REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
