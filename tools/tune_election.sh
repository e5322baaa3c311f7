#!/bin/bash
# Times every tools/variants/libmraft_hip_*.so on bench_election.py (GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune_el
for rep in $(seq 1 ${REPS:-2}); do
for lib in tools/variants/libmraft_hip_*.so; do
  tag=$(basename "$lib" .so); tag=${tag#libmraft_hip_}
  MRAFT_LIB="$PWD/$lib" timeout -k 10 120 python bench_election.py --no-cpu-baseline > gpurun_out/tune_el/$tag.$rep.json 2> gpurun_out/tune_el/$tag.$rep.err || { echo "$tag FAILED"; tail -3 gpurun_out/tune_el/$tag.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/tune_el/$tag.$rep.json')); print('$tag', round(d['roofline']['kernel_ms_mean']*1e3,1), 'us')"
done; done
