#!/bin/bash
# Round 3, call G: fold parity after the merged probe + launch changes, the
# fold variants on the message path (tools/tune_items.sh), and the 32,768-group
# tick trace with the XCD bits decoded.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3g
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_message_path_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/fold_tests.txt" 2>&1 || { echo "FAILED tests"; tail -30 "$OUT/fold_tests.txt"; exit 1; }
tail -2 "$OUT/fold_tests.txt"
REPS=2 VARIANTS="f*" bash tools/tune_items.sh || exit 1
TRACE_G=32768 TRACE_SAVE=$OUT/trace_g32768.npy MRAFT_LIB=$PWD/tools/variants/libmraft_hip_trace.so \
  timeout -k 10 180 python3 -u tools/trace_tick.py > "$OUT/trace_g32768.txt" 2>&1 || { echo "FAILED trace"; tail -5 "$OUT/trace_g32768.txt"; exit 1; }
head -14 "$OUT/trace_g32768.txt"
