#!/bin/bash
# Tick-kernel A/B with traffic (GPU box): for every tools/variants/libmraft_hip_<tag>.so
# named in LIBS (default: all) and the in-tree library, REPS interleaved timed
# bench lines (--no-secondary) and one FETCH_SIZE and one WRITE_SIZE pass each;
# tools/ab_tick_pmc.py prints per-step HBM bytes (calibrated like
# profiles/pmc_traffic_s2.json) beside the kernel time.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abtick}
mkdir -p "$OUT"
libs="${LIBS:-$(cd tools/variants && ls libmraft_hip_*.so | sed 's/libmraft_hip_//; s/\.so$//')} in-tree"
ARGS="--no-secondary --no-cpu-baseline ${BENCH_EXTRA:-}"
for rep in $(seq 1 ${REPS:-2}); do
  for t in $libs; do
    if [ "$t" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$t.so; fi
    timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 2 $ARGS > "$OUT/$t.$rep.json" 2> "$OUT/$t.$rep.err" \
      || { echo "$t bench failed"; tail -3 "$OUT/$t.$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$t.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$t', $rep, round(d['ms_per_step'],4), round(r['kernel_ms_mean'],4), round(r['frac'],3))"
  done
done
for t in $libs; do
  if [ "$t" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$t.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${t}_$c" -o p -- python3 bench.py --steps 5 --warmup 1 $ARGS \
      > "$OUT/pmc_${t}_$c.json" 2> "$OUT/pmc_${t}_$c.err" || { echo "$t $c failed"; tail -3 "$OUT/pmc_${t}_$c.err"; exit 1; }
  done
done
unset MRAFT_LIB
python3 tools/ab_tick_pmc.py "$OUT" $libs | tee "$OUT/summary.json"
