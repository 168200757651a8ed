set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread -k "jointjerk or user_cost or callback" > gpurun_out/r4_dropin2.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v --timeout 300 --timeout-method thread -k "frontdoor_single or dynamic_problem_assignment" > gpurun_out/r4_dropin3.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
