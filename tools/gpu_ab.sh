#!/bin/bash
# A/B of tools/variants/*.so on the same state copies (tools/ab_variants.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
COPIES=${COPIES:-8} REPS=${REPS:-2} timeout -k 10 600 python tools/ab_variants.py > gpurun_out/ab.txt 2>&1; rc=$?; grep -v "^/opt" gpurun_out/ab.txt | tail -8; exit $rc
