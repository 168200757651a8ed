#!/bin/bash
# Round 5: host-loop bench line (config HB, batch 64) after the grouped launches, then suite part B.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_final
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python3 -u bench.py --config HB --batch 64 --steps 1 --warmup 0 > gpurun_out/prof_final/r05_bench_HB64b.json \
  2> gpurun_out/prof_final/r05_bench_HB64b.err
echo "HB rc=$?"
cat gpurun_out/prof_final/r05_bench_HB64b.json
bash tools/r5_suite.sh B
