# round 4: part-a failures with the calibrated envelope test
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 1100 python -u -m pytest tests/test_gpu.py -m gpu -v -s --timeout 900 --timeout-method thread -k "cartpose_tolerance_cnt or test_full_batch_every_problem" > gpurun_out/r4_g21.log 2>&1
rc=$?
cp gpurun_out/parity_table.json gpurun_out/r4_parity_table_g21.json 2>/dev/null
exit $rc
