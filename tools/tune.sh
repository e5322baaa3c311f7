#!/bin/bash
# Times every tools/variants/libmraft_hip_*.so on the headline bench (GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
for lib in tools/variants/libmraft_hip_*.so; do
  tag=$(basename "$lib" .so); tag=${tag#libmraft_hip_}
  MRAFT_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/tune/$tag.json 2> gpurun_out/tune/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/tune/$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/tune/$tag.json')); r=d['roofline']; print('$tag', round(r['kernel_ms_mean']*1e3,1), 'us', round(r['frac'],3))"
done
