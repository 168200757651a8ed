# A/B of the generic-step build's d-value / middle-block phase (THIP_GEN_DV_HOIST):
# phase profile of config HA on the working build (PP_ROOT=r6dv0: the build
# without it), then the working build against the main build's generic step
# (bitwise), run via gpurun
set -e
L=gpurun_out/dv_ab.log
: > $L
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python3 -u tools/phase_profile.py HA 512 > gpurun_out/pp_HA_new.txt 2>&1
timeout -k 10 300 python3 -u tools/gen_ab.py HA 512 >> $L 2>&1
timeout -k 10 300 python3 -u tools/gen_ab.py E 64 >> $L 2>&1
