#!/bin/bash
# Kernel trace of the message-level path (tools/bench_items.py): per-kernel
# stats and the timeline gaps inside one handle call.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-dev}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/items -o items -- python3 tools/bench_items.py > gpurun_out/items_prof.json 2> gpurun_out/items_prof.err &&
cp "$(find gpurun_out/prof/items -name 'items_kernel_stats.csv' | head -1)" gpurun_out/${TAG}_items_kernel_stats.csv &&
cp "$(find gpurun_out/prof/items -name 'items_kernel_trace.csv' | head -1)" gpurun_out/${TAG}_items_kernel_trace.csv &&
python3 tools/items_timeline.py gpurun_out/${TAG}_items_kernel_trace.csv
