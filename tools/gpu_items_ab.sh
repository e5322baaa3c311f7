#!/bin/bash
# Message-level path (tools/bench_items.py) per tools/variants library, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in tools/variants/libmraft_hip_*.so; do
    t=$(basename $v .so); t=${t#libmraft_hip_}
    MRAFT_LIB=$PWD/$v timeout -k 10 300 python tools/bench_items.py > gpurun_out/items_${t}_$r.json 2> gpurun_out/items_${t}_$r.err || exit 1
    echo "$t $r $(python3 -c "import json;d=json.load(open('gpurun_out/items_${t}_$r.json'));print(d['ms_per_call'], d['roofline']['frac'], d['fused_tick_ms'])")"
  done
done
