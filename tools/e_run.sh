# config E checks on the GPU box: dual-arm parity tests, then the phase profile
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 500 --timeout-method thread -k "dual_arm" > gpurun_out/e_tests.log 2>&1
timeout -k 10 200 python -u tools/phase_profile.py E 16 > gpurun_out/e_phase.txt 2>&1
