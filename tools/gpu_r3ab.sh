#!/bin/bash
# Round 3, call AB: the driver's round-end sequence on the final round-3 tree
# as rebuilt in a fresh container: pytest -m gpu, smoke(), the default bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_v13}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/gpu_tests.txt" | head -20; tail -20 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { echo "FAILED smoke"; tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 500 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "FAILED bench"; tail -10 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))
s=d.get('secondary',{})
for k in ('message_path_config3','config4_one_gpu'):
    v=s.get(k,{}); print(k, {x: v.get(x) for x in ('ms_per_step','gather_ms','handle_ms','fold_ms','value') if x in v})
"
echo done
