#!/bin/bash
# Round 3, call AA: the AppendEntries plan's sets in eight lists (one counter
# per list instead of one counter for every plan workgroup's atomic) — GPU
# parity of the message path and the handle call, A/B against HEAD on the
# config #3 message path, and a kernel trace of the new library's path.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3aa
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py tests/test_sim_many.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
REPS=3 VARIANTS="*" PROFILE=1 bash tools/tune_items.sh > "$OUT/ab.txt" 2>&1 || { echo "FAILED ab"; tail -20 "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt" | cut -c1-200
echo done
