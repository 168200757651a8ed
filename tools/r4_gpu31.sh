# round 4: torso_arm_8dof_C repeated on the previous and the current build
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python3 -u tools/torso_repeat.py prevcmp 6 > gpurun_out/r4_g31_prev.log 2>&1
timeout -k 10 200 python3 -u tools/torso_repeat.py . 6 > gpurun_out/r4_g31_now.log 2>&1
