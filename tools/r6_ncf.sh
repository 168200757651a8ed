#!/bin/bash
# Round 6: contraction off + explicit fma in the segment (r6ncf) against the
# shipped build (.) and contraction off alone (r6nc): config C lone batch,
# torso_arm_8dof_C, parity sample.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_ncf.log
: > $L
timeout -k 10 200 python3 -u tools/c_ab.py . base 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r6ncf ncf 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r6nc nc 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 150 python3 -u tools/torso_repeat.py r6ncf 1 >> $L 2>&1 || exit 1
PARITY_ROOTS=".:r6ncf" timeout -k 10 500 python3 -u tools/parity.py C 512 B 256 A 256 >> $L 2>&1 || exit 1
cat $L
