#!/bin/bash
# Round 5: generic-path drop-ins beyond the fused caps, the host-loop worker pool,
# and the per-QP traces behind the round-4 spread excusals (numerical_ik1,
# arm_6dof_A problem 0, D-rank7 problem 837 = config C seed 8005).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dropin.py \
  tests/test_gpu_sco.py -k "long_horizon or second_jointvel or large_scene or numerical_ik1 or worker_pool" \
  > gpurun_out/r5_dropin.log 2>&1
rc=$?
timeout -k 10 200 python -u tools/hostloop_trace.py tests/golden/json/numerical_ik1.json > gpurun_out/r5_trace_ik1.txt 2>&1 &&
timeout -k 10 200 python -u tools/trace_compare.py arm_6dof_A 0 > gpurun_out/r5_trace_arm6.txt 2>&1 &&
timeout -k 10 200 python -u tools/trace_compare.py C@8005 0 > gpurun_out/r5_trace_d837.txt 2>&1
rc2=$?
echo "rc=$rc rc2=$rc2"
tail -12 gpurun_out/r5_dropin.log; tail -4 gpurun_out/r5_trace_ik1.txt gpurun_out/r5_trace_arm6.txt gpurun_out/r5_trace_d837.txt
