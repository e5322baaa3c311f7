#!/bin/bash
# Full GPU-box pass: parity suite, profile (trace + calibrated PMC), summary into
# profiles/<TAG>_*, then the headline bench with the fresh traffic figure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-dev}
mkdir -p gpurun_out
echo "== pytest -m gpu" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } &&
echo "== profile" && bash tools/profile_round.sh > gpurun_out/profile.log 2>&1 &&
python tools/pmc_summary.py "$TAG" > gpurun_out/pmc_summary.log 2>&1 && cp profiles/pmc_traffic.json profiles/${TAG}_*.csv gpurun_out/ &&
echo "== bench" && { timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -2 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ]; } &&
echo "== microbench" && { timeout -k 5 120 ./tools/mb_segcopy > gpurun_out/mb_segcopy.txt 2>&1; rc=$?; cat gpurun_out/mb_segcopy.txt; [ $rc -eq 0 ]; } &&
echo "== election storm (config #5)" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/el -o el -- python3 bench_election.py --no-cpu-baseline > gpurun_out/prof/el_bench.json 2> gpurun_out/prof/el_bench.err &&
cp "$(find gpurun_out/prof/el -name 'el_kernel_stats.csv' | head -1)" gpurun_out/${TAG}_election_kernel_stats.csv &&
timeout -k 10 300 python bench_election.py > gpurun_out/${TAG}_election_bench.json 2> gpurun_out/election_bench.err && cat gpurun_out/${TAG}_election_bench.json &&
echo "== message path" &&
timeout -k 10 300 python tools/bench_items.py > gpurun_out/${TAG}_message_path.json 2> gpurun_out/items.err && cat gpurun_out/${TAG}_message_path.json
