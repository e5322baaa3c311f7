#!/bin/bash
# Round 3, call N: the reply fold's per-segment timeline (diagnostic build).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3n
mkdir -p "$OUT"
MRAFT_LIB=$PWD/tools/variants/libmraft_hip_ftrace.so timeout -k 10 300 python3 -u tools/trace_fold.py > "$OUT/trace_fold.txt" 2>&1 || { echo "FAILED"; tail -10 "$OUT/trace_fold.txt"; exit 1; }
cat "$OUT/trace_fold.txt"
