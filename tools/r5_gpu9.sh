#!/bin/bash
# Round 5: the generic QP solver's wave-parallel / one-wave-chain KKT solve:
# host-loop batch timing with the KKT shape, then the generic-path GPU tests.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python -u tools/hb_probe.py 1 8 > gpurun_out/r5_hb_probe3.log 2>&1
rc=$?
cat gpurun_out/r5_hb_probe3.log
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=0 -m gpu \
  tests/test_gpu_sco.py tests/test_gpu_tsqp.py tests/test_gpu_dropin.py > gpurun_out/r5_generic_tests.log 2>&1
echo "tests rc=$?"
grep -E "PASSED|FAILED|ERROR|passed|failed|s call" gpurun_out/r5_generic_tests.log | tail -80
