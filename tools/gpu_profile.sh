#!/bin/bash
# Profile + headline bench + secondary benches on a GPU box (no test suite):
# kernel trace, calibrated FETCH/WRITE traffic (tools/profile_round.sh +
# pmc_summary.py -> profiles/<TAG>_*), bench.py with the fresh traffic figure,
# the election storm and the message-level path. Results land in gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-dev}
mkdir -p gpurun_out
echo "== profile" && bash tools/profile_round.sh > gpurun_out/profile.log 2>&1 &&
python tools/pmc_summary.py "$TAG" > gpurun_out/pmc_summary.log 2>&1 && cp profiles/pmc_traffic.json profiles/${TAG}_*.csv gpurun_out/ &&
echo "== bench" && { timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ]; } &&
echo "== election storm (config #5)" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/el -o el -- python3 bench_election.py --no-cpu-baseline > gpurun_out/prof/el_bench.json 2> gpurun_out/prof/el_bench.err &&
cp "$(find gpurun_out/prof/el -name 'el_kernel_stats.csv' | head -1)" gpurun_out/${TAG}_election_kernel_stats.csv &&
timeout -k 10 300 python bench_election.py > gpurun_out/${TAG}_election_bench.json 2> gpurun_out/election_bench.err && cat gpurun_out/${TAG}_election_bench.json &&
echo "== message path" &&
timeout -k 10 300 python tools/bench_items.py > gpurun_out/${TAG}_message_path.json 2> gpurun_out/items.err && cat gpurun_out/${TAG}_message_path.json
