#!/bin/bash
# Round 3, call Q: the reply fold with its a1 scans in a second launch
# (k_fold_scan), on top of the spill-free handler — parity (message path,
# ring, scenario replays on one group and on many), A/B against HEAD and the
# scan kernel's knobs on the config #3 message path, per-kernel HBM traffic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3q
mkdir -p "$OUT"
export MRAFT_SIM_PROGRESS=1000
timeout -k 10 900 python3 -u -m pytest tests/test_message_path_gpu.py tests/test_gpu_parity.py tests/test_ring.py tests/test_sim2b.py tests/test_sim_many.py -m gpu -x -q -s \
  --timeout 800 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "FAILED tests"; grep -E "FAILED|Error|assert" "$OUT/tests.txt" | head -20; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
REPS=3 VARIANTS="*" bash tools/tune_items.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  STEPS=4 timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o p -- python3 tools/bench_items.py > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.err; exit 1; }
done
echo done
