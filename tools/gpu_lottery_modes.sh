#!/bin/bash
# Slow-copy population under (a) no profiler, (b) rocprofv3 kernel trace,
# (c) rocprofv3 --pmc with one cheap counter (GRBM_GUI_ACTIVE).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lm
echo "== plain" && COPIES=10 timeout -k 10 300 python3 tools/exp_lottery_pmc.py > gpurun_out/lm/plain.txt 2>&1 && grep "^pass" gpurun_out/lm/plain.txt | tr '\n' ' ' | head -c 3000; echo
echo "== kernel-trace" && COPIES=10 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lm/kt -o kt -- python3 tools/exp_lottery_pmc.py > gpurun_out/lm/kt.txt 2>&1 && grep "^pass" gpurun_out/lm/kt.txt | tr '\n' ' ' | head -c 3000; echo
echo "== pmc GRBM_GUI_ACTIVE" && COPIES=10 timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lm/pmc -o pmc -- python3 tools/exp_lottery_pmc.py > gpurun_out/lm/pmc.txt 2>&1 && grep "^pass" gpurun_out/lm/pmc.txt | tr '\n' ' ' | head -c 3000; echo
find gpurun_out/lm -name "*.csv" | head
