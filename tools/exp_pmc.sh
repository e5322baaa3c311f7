#!/bin/bash
# Traffic experiment (GPU box): for every tools/variants/libmraft_hip_<tag>.so,
# the tick's kernel time (bench) and FETCH_SIZE / WRITE_SIZE (separate --pmc
# passes), summarised by tools/exp_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${EXTRA_ARGS:-}"
for lib in tools/variants/libmraft_hip_*.so; do
  tag=$(basename "$lib" .so); tag=${tag#libmraft_hip_}
  export MRAFT_LIB="$PWD/$lib"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${EXTRA_ARGS:-} > $O/$tag.json 2> $O/$tag.err || { echo "$tag bench FAILED"; tail -3 $O/$tag.err; exit 1; }
  for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/${tag}_$c -o p -- python3 bench.py $ARGS > /dev/null 2> $O/${tag}_$c.err || { echo "$tag $c FAILED"; tail -3 $O/${tag}_$c.err; exit 1; }
  done
  echo "$tag done"
done
python tools/exp_summary.py $O
