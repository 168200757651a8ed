# A/B of the generic QP kernel's pass-scheduled forward solve (config HB), run via gpurun
set -e
mkdir -p gpurun_out
L=gpurun_out/hb_ab.log
: > $L
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
B=${1:-16}
THIP_QP_LEVEL_SOLVE=1 timeout -k 10 400 python3 -u tools/hb_ab.py run level $B >> $L 2>&1
timeout -k 10 400 python3 -u tools/hb_ab.py run pass $B >> $L 2>&1
python3 tools/hb_ab.py compare level pass >> $L 2>&1
