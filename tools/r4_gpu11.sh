# round 4: traces and contact rows of the round-3 build and the current one (config C continuous).
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
set -e
timeout -k 10 300 python -u tools/r3_trace.py "$PWD/r3cmp" r3 > gpurun_out/r4_g11_r3.log 2>&1
timeout -k 10 300 python -u tools/r3_trace.py "$PWD" now > gpurun_out/r4_g11_now.log 2>&1
