#!/bin/bash
# Round 5: config E bench line (512 problems per GPU, three batches in flight).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python3 -u bench.py --config E --batch 512 --inflight 3 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/r5_bench_E.json 2> gpurun_out/r5_bench_E.err
echo "E rc=$?"
cat gpurun_out/r5_bench_E.json
