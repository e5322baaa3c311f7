#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lp
echo "== utcl1 pass" && COPIES=12 timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum --output-format csv -d gpurun_out/lp/a -o a -- python3 tools/exp_lottery_pmc.py > gpurun_out/lp/a.txt 2>&1; rc=$?; tail -3 gpurun_out/lp/a.txt; [ $rc -eq 0 ] &&
echo "== tcc pass" && COPIES=12 timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum --output-format csv -d gpurun_out/lp/b -o b -- python3 tools/exp_lottery_pmc.py > gpurun_out/lp/b.txt 2>&1; rc=$?; tail -3 gpurun_out/lp/b.txt; [ $rc -eq 0 ] &&
find gpurun_out/lp -name "*counter_collection.csv"
