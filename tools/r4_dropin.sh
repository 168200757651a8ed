# round 4: the drop-in tests (host loop + device-evaluated terms), then the bench line
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_dropin.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
