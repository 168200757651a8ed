# round 4: per-QP trace of torso_arm_8dof_C problem 2, current build
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python3 -u tools/trace_compare.py torso_arm_8dof_C 2 > gpurun_out/r4_g33_trace.log 2>&1
