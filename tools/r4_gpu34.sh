# round 4: torso_arm_8dof_C on two variant builds (a.x recomputed in the update / row-major back-substitution)
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
for t in var_noHG var_oldBS; do
  timeout -k 10 200 python3 -u tools/torso_repeat.py $t 1 > gpurun_out/r4_g34_$t.log 2>&1 || exit $?
done
