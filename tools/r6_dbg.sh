#!/bin/bash
# Round 6: (1) per-ADMM-iteration dumps of torso_arm_8dof_C problem 2, QP 6, from
# the shipped source and from the a.x reuse (tools/r6_dbg_apply.py trees);
# (2) parity sample of the -ffp-contract=off build against the shipped one;
# (3) last: the 1,024-thread generic-step build with workspace-pointer checks
# (tools/r6_bounds_apply.py) on config C x4 -- may fault, so it runs last.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_dbg.log
: > $L
export THIP_DBG_PROB=2 THIP_DBG_QP=6
THIP_DBG_OUT=gpurun_out/dbg_base.bin timeout -k 10 150 python3 -u tools/torso_repeat.py r6dbgbase 1 >> $L 2>&1 || exit 1
THIP_DBG_OUT=gpurun_out/dbg_ax.bin timeout -k 10 150 python3 -u tools/torso_repeat.py r6dbgax 1 >> $L 2>&1 || exit 1
unset THIP_DBG_PROB THIP_DBG_QP
PARITY_ROOTS=".:r6nc" timeout -k 10 400 python3 -u tools/parity.py C 256 B 128 A 128 C-cont 64 >> $L 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/gen_ab.py C 4 0 r6g1024 > gpurun_out/r6_g1024.log 2>&1
echo "gen_ab 1024 exit $?" >> $L
cat $L
