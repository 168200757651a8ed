# round 4 full GPU suite, part a: tests/test_gpu.py (no -x: every failure is listed)
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 1100 python -u -m pytest tests/test_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r4_suite_a.log 2>&1
rc=$?
cp gpurun_out/parity_table.json gpurun_out/r4_parity_table_a.json 2>/dev/null
exit $rc
