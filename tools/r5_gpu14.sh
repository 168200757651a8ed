#!/bin/bash
# Round 5: the host-loop bench line (config HB) at batch 64.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_final
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 700 python3 -u bench.py --config HB --batch 64 --steps 1 --warmup 0 > gpurun_out/prof_final/r05_bench_HB64.json \
  2> gpurun_out/prof_final/r05_bench_HB64.err
echo "HB rc=$?"
cat gpurun_out/prof_final/r05_bench_HB64.json
