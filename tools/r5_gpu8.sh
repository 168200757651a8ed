#!/bin/bash
# Round 5: the a.x-reuse bisection, second set (r5v7: a barrier before the
# hinge loop; r5v8: only the hinge's step index loaded, unused; r5v9: only the
# hinge coefficients loaded, unused), then where a host-loop batch spends its time.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L2=gpurun_out/r5_ax_bisect2.log
: > $L2
for v in r5v7 r5v8 r5v9; do
  timeout -k 10 120 python -u tools/torso_repeat.py $v 1 >> $L2 2>&1 || { echo "FAILED $v" >> $L2; cat $L2; exit 1; }
done
cat $L2
timeout -k 10 400 python -u tools/hb_probe.py 1 8 32 > gpurun_out/r5_hb_probe.log 2>&1
echo "probe rc=$?"
cat gpurun_out/r5_hb_probe.log
