#!/bin/bash
# Round 5: the generic QP kernel with in-order batched row sums on the LDS-staged factor.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python -u tools/hb_probe.py 1 > gpurun_out/r5_hb_probe5.log 2>&1
rc=$?
cat gpurun_out/r5_hb_probe5.log
exit $rc
