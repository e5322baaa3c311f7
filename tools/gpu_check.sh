#!/bin/bash
# One GPU-box validation pass (run via gpurun from the repo root): smoke, the
# GPU parity suite, then the headline bench (optionally under rocprofv3
# kernel trace). Every GPU step has its own time limit and the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
echo "== pytest -m gpu" && { timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } &&
echo "== bench" && { timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 4} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ]; } &&
if [ -n "$KTRACE" ]; then
  echo "== kernel trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o kt -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kt_bench.json 2> gpurun_out/kt_bench.err && cat gpurun_out/kt/kt_kernel_stats.csv
fi
