#!/bin/bash
# Round 3, call A: where the ~20 us per-step gap of the fan-in runs comes from
# (VERDICT r2 weak #3). 32,768 groups per GPU (config #4's N = 8 shard):
#   legacy  round 2's markers (start + end per tick + the ABI's fan-in event)
#   chain   one marker per tick shared by timing and the fan-in wait
#   nofan   no fan-in, one marker per tick
#   extra3  no fan-in, three extra untimed markers per tick
# then a kernel trace of the chain run (the dispatch gaps between ticks).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3a
mkdir -p "$OUT"
B="python3 -u bench.py --global-groups 32768 --steps 30 --warmup 3 --no-cpu-baseline --no-secondary"
run() {  # name, extra args
  echo "== $1"
  timeout -k 10 180 $B ${@:2} > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "FAILED $1 rc=$?"; tail -5 "$OUT/$1.err"; exit 1; }
  python3 - "$OUT/$1.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, c = d["roofline"], d["config"]
print(f'  step {d["ms_per_step"]:.4f} ms  kernel {r["kernel_ms_mean"]:.4f} (min {r["kernel_ms_min"]:.4f})  '
      f'gap {c["step_minus_kernel_ms"] * 1e3:.1f} us  frac {r["frac"]:.3f}  ag {c["allgather_ms_mean"]}')
EOF
}
run legacy --fanin-at-1 --fanin-marks legacy
run chain --fanin-at-1
run nofan
run extra3 --extra-marks 3
run legacy2 --fanin-at-1 --fanin-marks legacy
run chain2 --fanin-at-1
echo "== kernel trace (chain)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
  python3 bench.py --global-groups 32768 --steps 30 --warmup 3 --no-cpu-baseline --no-secondary --fanin-at-1 \
  > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || { echo "FAILED trace"; tail -5 "$OUT/kt_bench.err"; exit 1; }
echo "== done"
