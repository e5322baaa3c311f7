#!/bin/bash
# GPU parity suite, then the A/B of tools/variants on the same state copies.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
echo "== ab" && COPIES=${COPIES:-8} REPS=${REPS:-2} timeout -k 10 600 python tools/ab_variants.py > gpurun_out/ab.txt 2>&1; rc=$?; grep -v "^/opt" gpurun_out/ab.txt | tail -8; exit $rc
