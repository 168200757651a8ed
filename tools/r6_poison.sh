#!/bin/bash
# Round 6: NaN-poisoned workspace and LDS (tools/r6_poison_apply.py) on the
# shipped source (r6pz) and with the a.x reuse (r6pzax): torso_arm_8dof_C, then
# a parity sample of r6pz against the shipped build (identical results = no
# read of unwritten memory reaches them); the reuse build alone / static; last
# the 1,024-thread build with a larger ROCr scratch limit (may fault).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_poison.log
: > $L
for t in r6pz r6pzax; do
  timeout -k 10 150 python3 -u tools/torso_repeat.py $t 2 >> $L 2>&1 || exit 1
done
timeout -k 10 150 python3 -u tools/torso_repeat.py r6ax 1 2 >> $L 2>&1 || exit 1
timeout -k 10 150 python3 -u tools/torso_repeat.py r6ax 1 2 static >> $L 2>&1 || exit 1
PARITY_ROOTS=".:r6pz" timeout -k 10 500 python3 -u tools/parity.py C 256 B 128 A 128 C-cont 64 J 64 C-disc 64 E 8 >> $L 2>&1 || exit 1
HSA_SCRATCH_SINGLE_LIMIT=8589934592 timeout -k 10 120 python3 -u tools/gen_ab.py C 4 0 r6g1024 > gpurun_out/r6_g1024b.log 2>&1
echo "gen_ab 1024 (scratch limit 8 GB) exit $?" >> $L
cat $L
