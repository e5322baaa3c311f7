#!/bin/bash
# Round 3, call K: where the reply fold's time goes (timing-only variants:
# no a1 log reads / probes only) and the message path's PMC traffic per
# kernel (separate FETCH_SIZE / WRITE_SIZE passes + calibration).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=2 VARIANTS="i*" bash tools/tune_items.sh || exit 1
OUT=gpurun_out/r3k
mkdir -p "$OUT"
STEPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 tools/bench_items.py > "$OUT/kt.json" 2> "$OUT/kt.err" || { echo "FAILED kt"; tail -5 "$OUT/kt.err"; exit 1; }
STEPS=4 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 tools/bench_items.py > "$OUT/fetch.json" 2> "$OUT/fetch.err" || { echo "FAILED fetch"; tail -5 "$OUT/fetch.err"; exit 1; }
STEPS=4 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 tools/bench_items.py > "$OUT/write.json" 2> "$OUT/write.err" || { echo "FAILED write"; tail -5 "$OUT/write.err"; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/cal_fetch" -o calf -- ./tools/calib_pmc > "$OUT/calib.json" || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/cal_write" -o calw -- ./tools/calib_pmc > /dev/null || exit 1
echo done
