#!/bin/bash
# Round 3, call Y: the N > 1 bench path with the RCCL data-path fan-in, two
# ranks sharing the one GPU of this box (an 8-GPU node is not available to
# builder runs): ncclCommInitRank with nranks = 2 through mraft_comm_init, the
# unique-id handoff over gloo, the per-step check of the gathered words
# against the per-rank exports. RCCL may refuse two ranks on one device; the
# run records what happens either way.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3y
mkdir -p "$OUT"
NCCL_DEBUG=WARN timeout -k 10 240 python3 -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench2_rccl.json" 2> "$OUT/bench2_rccl.err"
echo "rc=$?"
grep -iE "duplicate|WARN|invalid" "$OUT/bench2_rccl.err" | head -20 || true
cat "$OUT/bench2_rccl.json"
