#!/bin/bash
# Round 5 final check, as the driver runs it: the whole -m gpu suite in one
# session (per-test wall times), then smoke().
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
THIP_TEST_TIMES=1 timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r5_final_suite.log 2>&1
rc=$?
echo "suite rc=$rc"
tail -3 gpurun_out/r5_final_suite.log
cp gpurun_out/parity_table.json gpurun_out/r5_final_parity_table.json 2>/dev/null
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final_smoke.log 2>&1
echo "smoke rc=$?"
tail -2 gpurun_out/r5_final_smoke.log
