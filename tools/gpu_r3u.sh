#!/bin/bash
# Round 3, call U: the reply fold generalised to 64/GW segments per wave (GW
# lanes each: 4 x 16 by default, fg8 = 8 x 8), the pending-scan marker as one
# 8-B write, the plan's totals published by the handler — parity (fold,
# message path, ring, scenario replays on one group and on many), A/B against
# m8 on the config #3 message path, kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3u
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=1000
timeout -k 10 900 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py tests/test_ring.py tests/test_sim2b.py tests/test_sim_many.py -m gpu -x -q -s \
  --timeout 800 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
PROFILE=1 REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
