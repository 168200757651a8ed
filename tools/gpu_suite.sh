# the whole -m gpu suite on the GPU box, then smoke(); progress ticker for the idle-output watchdog
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
THIP_TEST_TIMES=1 timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --durations=40 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
