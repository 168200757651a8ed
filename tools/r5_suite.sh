#!/bin/bash
# Round 5: the -m gpu suite in two parts (A: test_gpu.py, B: the rest) with
# per-test durations; the parity table of the session is written by conftest.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PART=${1:-A}
KSEL=()
[ -n "$2" ] && KSEL=(-k "$2")
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
if [ "$PART" = A ]; then
  FILES="tests/test_gpu.py"
else
  FILES=$(ls tests/test_gpu*.py | grep -v "tests/test_gpu.py")
fi
THIP_TEST_TIMES=1 timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread --durations=30 -m gpu $FILES "${KSEL[@]}" \
  > gpurun_out/r5_suite_$PART.log 2>&1
rc=$?
cp gpurun_out/parity_table.json gpurun_out/r5_parity_table_$PART.json 2>/dev/null
echo "suite $PART rc=$rc"
grep -E "FAILED|ERROR|passed|failed|[0-9]s call" gpurun_out/r5_suite_$PART.log | head -40
exit $rc
