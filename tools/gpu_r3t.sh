#!/bin/bash
# Round 3, call T: the a1 scans with four ranges in flight per wave
# (k_fold_scan4), the gather's slot words in one round trip, the plan's totals
# published by the handler's first workgroup — parity (fold, message path,
# ring, scenario replays on one group and on many), A/B against m8 (the
# previous default) on the config #3 message path, kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3t
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=1000
timeout -k 10 900 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py tests/test_ring.py tests/test_sim2b.py tests/test_sim_many.py -m gpu -x -q -s \
  --timeout 800 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
PROFILE=1 REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
