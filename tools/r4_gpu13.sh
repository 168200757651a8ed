# round 4: bisect the config C continuous regression -- rows builder (A) and scan passes (B) at their round-3 form.
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
set -e
timeout -k 10 300 python -u tools/r3_ccont.py "$PWD/r4var/A" > gpurun_out/r4_g13_A.log 2>&1
timeout -k 10 300 python -u tools/r3_ccont.py "$PWD/r4var/B" > gpurun_out/r4_g13_B.log 2>&1
