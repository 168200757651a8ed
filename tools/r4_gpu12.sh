# round 4: run-to-run determinism of the round-3 build and the current one (config C continuous).
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
set -e
timeout -k 10 300 python -u tools/determinism.py "$PWD/r3cmp" > gpurun_out/r4_g12_r3.log 2>&1
timeout -k 10 300 python -u tools/determinism.py "$PWD" > gpurun_out/r4_g12_now.log 2>&1
timeout -k 10 300 python -u tools/r3_ccont.py "$PWD/r4var/A" > gpurun_out/r4_g13_A.log 2>&1
timeout -k 10 300 python -u tools/r3_ccont.py "$PWD/r4var/B" > gpurun_out/r4_g13_B.log 2>&1
