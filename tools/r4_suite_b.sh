# round 4 full GPU suite, part b: every other -m gpu file, then smoke()
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread --ignore tests/test_gpu.py > gpurun_out/r4_suite_b.log 2>&1
rc=$?
cp gpurun_out/parity_table.json gpurun_out/r4_parity_table_b.json 2>/dev/null
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1
