#!/bin/bash
# Times every tools/variants/libmraft_hip_*.so on the headline bench (GPU box),
# REPS interleaved repetitions; prints mean and min tick-kernel time per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
for rep in $(seq 1 ${REPS:-2}); do
for lib in tools/variants/libmraft_hip_*.so; do
  tag=$(basename "$lib" .so); tag=${tag#libmraft_hip_}
  MRAFT_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline ${EXTRA_ARGS:-} \
      > gpurun_out/tune/$tag.$rep.json 2> gpurun_out/tune/$tag.$rep.err || { echo "$tag FAILED"; tail -3 gpurun_out/tune/$tag.$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/tune/$tag.$rep.json')); r=d['roofline']; print('$tag', round(r['kernel_ms_mean']*1e3,1), round(r['kernel_ms_min']*1e3,1), round(r['frac'],3))"
done; done
