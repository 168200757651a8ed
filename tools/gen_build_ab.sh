# round-6 A/B of the generic-step build (default for QPs outside the segment's
# domain) against the main build's generic step (tools/gen_ab.py), run via gpurun
set -e
L=gpurun_out/ab_gen.log
: > $L
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python3 -u tools/gen_ab.py HA 512 >> $L 2>&1
timeout -k 10 300 python3 -u tools/gen_ab.py E 64 >> $L 2>&1
timeout -k 10 200 python3 -u tools/gen_ab.py C 256 50 >> $L 2>&1
timeout -k 10 300 python3 -u tools/c_ab.py . now_C 1024 2 C >> $L 2>&1
timeout -k 10 600 python3 -u tools/parity.py B-acc 64 E 16 C50-cont 64 >> $L 2>&1
