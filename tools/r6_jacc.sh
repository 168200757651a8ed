#!/bin/bash
# Round 6: JointAccEqCost in the fused kernel -- the new GPU tests, then the
# shipped workloads bitwise against the previous commit's build (r6prev: the
# waypoint-pair generalisation must not move grp = 1 results).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_jacc.log
: > $L
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "joint_acc" >> $L 2>&1
echo "jacc tests exit $?" >> $L
timeout -k 10 300 python3 -u tools/build_bitwise.py r6prev prev >> $L 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/build_bitwise.py . now >> $L 2>&1 || exit 1
python3 tools/build_bitwise.py --compare prev now >> $L 2>&1
echo "bitwise exit $?" >> $L
