# round 4: bisect the torso_arm_8dof_C change over this round's commits
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
for t in bis_c7dfec2 bis_d62893d; do
  timeout -k 10 200 python3 -u tools/torso_repeat.py $t 1 > gpurun_out/r4_g32_$t.log 2>&1 || exit $?
done
