#!/bin/bash
# Round 5: a.x-reuse traces, per-pair collision GPU tests, generic-step build A/B on config E.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 100 python -u tools/ax_trace.py . head > gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 100 python -u tools/ax_trace.py r5ax2 reuse >> gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 100 python -u tools/ax_trace.py r5ax probe >> gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 300 python -u tools/gen_ab.py E 128 > gpurun_out/r5_gen_ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "pairs or dual_arm" > gpurun_out/r5_pairs.log 2>&1
rc=$?
echo "rc=$rc"
tail -4 gpurun_out/r5_axtrace.log; cat gpurun_out/r5_gen_ab.log; tail -15 gpurun_out/r5_pairs.log
exit $rc
