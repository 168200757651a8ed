#!/bin/bash
# Round 5: the generic QP kernel with its factor staged in LDS: host-loop batch
# timing, the generic-path GPU tests; then the a.x-reuse build (r5v1) with
# problem 2 alone and with static dispatch.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python -u tools/hb_probe.py 1 8 > gpurun_out/r5_hb_probe4.log 2>&1
rc=$?
cat gpurun_out/r5_hb_probe4.log
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=0 -m gpu \
  tests/test_gpu_sco.py tests/test_gpu_tsqp.py tests/test_gpu_dropin.py > gpurun_out/r5_generic_tests2.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "FAILED|ERROR|passed|failed|[0-9]s call" gpurun_out/r5_generic_tests2.log | head -30
[ $rc = 0 ] || exit $rc
L=gpurun_out/r5_ax_bisect3.log
: > $L
timeout -k 10 120 python -u tools/torso_repeat.py r5v1 1 2 >> $L 2>&1 && \
timeout -k 10 120 python -u tools/torso_repeat.py r5v1 1 2 static >> $L 2>&1 && \
timeout -k 10 120 python -u tools/torso_repeat.py r5v6 1 2 >> $L 2>&1
cat $L
