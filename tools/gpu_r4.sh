#!/bin/bash
# Round 4 GPU pass, parametrised: TAG names the output directory
# (gpurun_out/$TAG); STEPS lists what to run (tests, bench, prof, pmc, el).
#   TESTS   pytest selection (-k expression) for the tests step ("" = all -m gpu)
#   BENCH   extra bench.py arguments
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4_dev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for st in ${STEPS:-tests bench}; do
  case $st in
    tests)
      echo "== tests ${TESTS:-all}"
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; exit 1; } ;;
    bench)
      echo "== bench ${BENCH:-}"
      timeout -k 10 600 python3 -u bench.py ${BENCH:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; tail -4 "$OUT/bench.err"; [ $rc -eq 0 ] || exit 1
      python3 tools/summarize_bench.py "$OUT/bench.json" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done $TAG"
