#!/bin/bash
# Round 6: JointAccEqCost in the fused kernel after the coupling-array fix --
# GPU tests, then bench --config HA (config B + JointAcc, 1,024 problems).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r6_jacc2.log
: > $L
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "joint_acc" >> $L 2>&1
echo "jacc tests exit $?" >> $L
timeout -k 10 400 python3 -u bench.py --config HA --batch 1024 --steps 6 --warmup 1 > gpurun_out/r06_bench_HA.json 2> gpurun_out/r06_bench_HA.err
echo "bench HA exit $?" >> $L
