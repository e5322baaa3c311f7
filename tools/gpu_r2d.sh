#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lds in 0 8192 16384; do
  echo "== lds $lds" && MRAFT_TICK_DYN_LDS=$lds COPIES=10 timeout -k 10 300 python tools/exp_lottery3.py > gpurun_out/l3_$lds.txt 2>&1; rc=$?; tail -15 gpurun_out/l3_$lds.txt; [ $rc -eq 0 ] || exit $rc
done
