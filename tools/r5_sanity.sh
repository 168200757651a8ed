#!/bin/bash
# Round 5: final-tree sanity: smoke(), a short default bench, one generic-path GPU test.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_sanity_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r5_sanity_smoke.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/r5_sanity_bench.json 2> gpurun_out/r5_sanity_bench.err || exit 1
cut -c1-300 gpurun_out/r5_sanity_bench.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_dropin.py -k "prepared_hostloop or user_cost" > gpurun_out/r5_sanity_tests.log 2>&1
echo "tests rc=$?"
tail -1 gpurun_out/r5_sanity_tests.log
