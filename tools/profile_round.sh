#!/bin/bash
# Profiles the headline bench on a GPU box (run via gpurun from the repo root):
#   1. kernel trace + stats (per-kernel durations),
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (TCC slots: 3 + 2),
#   3. the same counters on tools/calib_pmc (known byte counts) for the
#      gfx950 width corrections of MI355X_MICROARCH.md §HBM.
# Outputs under gpurun_out/prof/; tools/pmc_summary.py turns them into
# profiles/<tag>_*.{csv,json,md}.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p "$OUT"
ARGS="--steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-}"
make -s -C tools
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py $ARGS > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err"
echo "== FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 bench.py $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
echo "== WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 bench.py $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
echo "== calibration"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/cal_fetch" -o calf -- ./tools/calib_pmc > "$OUT/calib.json"
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/cal_write" -o calw -- ./tools/calib_pmc > /dev/null
echo "== done"
find "$OUT" -name '*.csv' | head -50
