#!/bin/bash
# Round 6: -ffp-contract=off and the a.x reuse (tools/r6_ax_reuse.patch).
# Trees: . (shipped build), r6ax (reuse), r6nc (contraction off), r6ncax (both);
# built by tools/mktree.sh.  torso_arm_8dof_C twice per tree, config C and E
# lone-batch timing, a parity sample of every tree against one oracle run.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_fpc.log
: > $L
for t in . r6ax r6nc r6ncax; do
  timeout -k 10 150 python3 -u tools/torso_repeat.py $t 2 >> $L 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/c_ab.py . base 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r6nc nc 1024 3 >> $L 2>&1 || exit 1
python3 tools/c_ab.py --compare base nc >> $L 2>&1
for t in . r6nc r6ncax r6ax; do
  timeout -k 10 200 python3 -u tools/c_ab.py $t E_$(basename $t) 64 1 E >> $L 2>&1 || exit 1
done
PARITY_ROOTS=".:r6nc:r6ncax" timeout -k 10 400 python3 -u tools/parity.py C 256 B 128 A 128 C-cont 64 >> $L 2>&1 || exit 1
cat $L
