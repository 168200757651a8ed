# A/B of the generic QP kernel's forward solve (config HB), run via gpurun:
# level (THIP_QP_LEVEL_SOLVE=1: level by level, one thread per row) against
# pass (the default: passes of row segments); trajectories compared bitwise
set -e
mkdir -p gpurun_out
L=gpurun_out/hb_ab.log
: > $L
B=${1:-16}
THIP_QP_LEVEL_SOLVE=1 timeout -k 10 400 python3 -u tools/hb_ab.py run level $B >> $L 2>&1
timeout -k 10 400 python3 -u tools/hb_ab.py run pass $B >> $L 2>&1
python3 tools/hb_ab.py compare level pass >> $L 2>&1
