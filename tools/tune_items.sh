#!/bin/bash
# Times every tools/variants/libmraft_hip_*.so on tools/bench_items.py (GPU box),
# then a rocprofv3 kernel trace of the default library's message path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tune_items
for rep in $(seq 1 ${REPS:-2}); do
for lib in tools/variants/libmraft_hip_${VARIANTS:-*}.so; do
  tag=$(basename "$lib" .so); tag=${tag#libmraft_hip_}
  MRAFT_LIB="$PWD/$lib" STEPS=10 timeout -k 10 200 python tools/bench_items.py > gpurun_out/tune_items/$tag.$rep.json 2> gpurun_out/tune_items/$tag.$rep.err || { echo "$tag FAILED"; tail -3 gpurun_out/tune_items/$tag.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/tune_items/$tag.$rep.json')); print('$tag', d['ms_per_call'])"
done; done
if [ -n "$PROFILE" ]; then
  STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_items -o items -- python3 tools/bench_items.py > gpurun_out/prof_items.json 2> gpurun_out/prof_items.err &&
  cat "$(find gpurun_out/prof_items -name 'items_kernel_stats.csv' | head -1)"
fi
