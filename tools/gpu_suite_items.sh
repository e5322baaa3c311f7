#!/bin/bash
# GPU parity suite, then the message-level path's kernel timeline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
bash tools/gpu_items_prof.sh && cat gpurun_out/items_prof.json
