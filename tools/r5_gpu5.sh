#!/bin/bash
# Round 5: bisection builds of the reverted a.x reuse on torso_arm_8dof_C
# (r5v1: device-scope fence before the barrier after the back-substitution;
# r5v3: global-typed HG accesses; r5v6: the recomputation's loads kept alive, unused).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/r5_ax_bisect.log
: > $L
for v in r5v1 r5v3 r5v6; do
  timeout -k 10 120 python -u tools/torso_repeat.py $v 1 >> $L 2>&1 || { echo "FAILED $v" >> $L; break; }
done
cat $L
