# config C checks on the GPU box: segment parity tests, then the phase profile
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 500 --timeout-method thread -k "test_sqp_parity or test_sqp_parity_collision" > gpurun_out/c_tests.log 2>&1
timeout -k 10 200 python -u tools/phase_profile.py C 1024 > gpurun_out/c_phase.txt 2>&1
