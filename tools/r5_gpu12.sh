#!/bin/bash
# Round 5: generic QP kernel, wave-cooperative in-order KKT solve on the LDS-staged
# factor: host-loop batch timing, then the generic-path GPU tests.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python -u tools/hb_probe.py 8 > gpurun_out/r5_hb_probe6.log 2>&1
rc=$?
cat gpurun_out/r5_hb_probe6.log
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=15 -m gpu \
  tests/test_gpu_sco.py tests/test_gpu_tsqp.py tests/test_gpu_dropin.py > gpurun_out/r5_generic_tests3.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "FAILED|ERROR|passed|failed|[0-9]s call" gpurun_out/r5_generic_tests3.log | head -30
exit $rc
