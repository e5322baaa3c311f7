#!/bin/bash
# round 2: message-level parity (new tests) + the placement experiment
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== message path tests" && timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_message_path_gpu.py > gpurun_out/msg_test.log 2>&1; rc=$?; tail -12 gpurun_out/msg_test.log; [ $rc -eq 0 ] &&
echo "== lottery" && COPIES=16 timeout -k 10 500 python tools/exp_lottery.py > gpurun_out/lottery.txt 2>&1; rc=$?; tail -24 gpurun_out/lottery.txt; exit $rc
