#!/bin/bash
# PMC traffic of the headline tick at every per-GPU shard size the bench uses
# (65,536 = config #3 / config #4 at N = 4; 32,768 at N = 8; 131,072 at N = 2;
# 262,144 = config #4 on one GPU), plus the kernel trace of the default bench
# line: separate --pmc passes (FETCH_SIZE, WRITE_SIZE), the gfx950 width
# corrections measured on tools/calib_pmc in the same run
# (MI355X_MICROARCH.md §HBM). Outputs under gpurun_out/pmc_<G>/; then
# `python tools/pmc_summary.py <tag>_g<G> gpurun_out/pmc_<G>` per size.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
[ -x tools/calib_pmc ] || { echo "tools/calib_pmc not built"; exit 1; }
for G in ${SIZES:-65536 32768 131072 262144}; do
  OUT=gpurun_out/pmc_$G
  mkdir -p "$OUT"
  ARGS="--global-groups $G --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-secondary"
  echo "== $G kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py $ARGS \
    > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || { echo "FAILED kt $G"; tail -5 "$OUT/kt_bench.err"; exit 1; }
  echo "== $G FETCH_SIZE"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 bench.py $ARGS \
    > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err" || { echo "FAILED fetch $G"; tail -5 "$OUT/fetch_bench.err"; exit 1; }
  echo "== $G WRITE_SIZE"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 bench.py $ARGS \
    > "$OUT/write_bench.json" 2> "$OUT/write_bench.err" || { echo "FAILED write $G"; tail -5 "$OUT/write_bench.err"; exit 1; }
  echo "== $G calibration"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/cal_fetch" -o calf -- ./tools/calib_pmc > "$OUT/calib.json" || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/cal_write" -o calw -- ./tools/calib_pmc > /dev/null || exit 1
done
echo "== done"
