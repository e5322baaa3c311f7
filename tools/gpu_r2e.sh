#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tick parity" && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_message_path_gpu.py -k "tick or message or long or stale or kat" > gpurun_out/tick_parity.log 2>&1; rc=$?; tail -3 gpurun_out/tick_parity.log; [ $rc -eq 0 ] &&
echo "== ab" && COPIES=${COPIES:-8} REPS=2 timeout -k 10 600 python tools/ab_variants.py > gpurun_out/ab.txt 2>&1; rc=$?; grep -v "^/opt" gpurun_out/ab.txt | tail -8; exit $rc
