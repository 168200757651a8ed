#!/bin/bash
# Round 5: the generic-step build at 512 threads on config E (32, 128, 512
# problems; stops at the first failure), the a.x-reuse bisection builds, and a
# short host-loop bench (config HB).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r5_gen_E.log
: > $L
for spec in "E 32 0" "E 128 0" "E 512 0"; do
  echo "=== $spec" >> $L
  timeout -k 10 300 python -u tools/gen_ab.py $spec >> $L 2>&1 || { echo "FAILED: $spec rc=$?" >> $L; cat $L; exit 1; }
done
cat $L
L2=gpurun_out/r5_ax_bisect.log
: > $L2
for v in r5v1 r5v3 r5v6; do
  timeout -k 10 120 python -u tools/torso_repeat.py $v 1 >> $L2 2>&1 || { echo "FAILED $v" >> $L2; cat $L2; exit 1; }
done
cat $L2
timeout -k 10 300 python -u bench.py --config HB --batch 256 --steps 2 --warmup 1 > gpurun_out/r5_hb.json 2> gpurun_out/r5_hb.err
echo "hb rc=$?"
cat gpurun_out/r5_hb.json; tail -5 gpurun_out/r5_hb.err
