set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== fanin test" && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fanin_gpu.py > gpurun_out/fanin_test.log 2>&1; rc=$?; tail -8 gpurun_out/fanin_test.log; [ $rc -eq 0 ] &&
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] &&
echo "== fanin at 1, cus 0" && timeout -k 10 300 python bench.py --fanin-at-1 --no-cpu-baseline > gpurun_out/fan0.json 2> gpurun_out/fan0.err; rc=$?; tail -2 gpurun_out/fan0.err; cat gpurun_out/fan0.json; [ $rc -eq 0 ] &&
echo "== fanin at 1, cus 8" && timeout -k 10 300 python bench.py --fanin-at-1 --fanin-cus 8 --no-cpu-baseline > gpurun_out/fan8.json 2> gpurun_out/fan8.err; rc=$?; tail -2 gpurun_out/fan8.err; cat gpurun_out/fan8.json; [ $rc -eq 0 ]
