#!/bin/bash
# Round 3, call B: the default one-GPU bench line (headline + secondaries +
# the new config #4 one-GPU anchor + affinity-based CPU baseline).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3b
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
tail -5 "$OUT/bench.err"
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'nproc', os.cpu_count()); print(open('/sys/fs/cgroup/cpu.max').read())" || true
