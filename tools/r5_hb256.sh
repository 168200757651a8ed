#!/bin/bash
# Round 5: the host-loop bench line (config HB) at batch 256.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 1000 python3 -u bench.py --config HB --batch 256 --steps 1 --warmup 0 > gpurun_out/r5_bench_HB256.json \
  2> gpurun_out/r5_bench_HB256.err
echo "HB rc=$?"
cut -c1-400 gpurun_out/r5_bench_HB256.json
