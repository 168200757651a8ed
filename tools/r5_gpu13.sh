#!/bin/bash
# Round 5: config C A/B (the chain solve's prefetch group 4 -> 8) and the
# host-loop bench line at batch 8.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_final
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r5_c_ab.log
: > $L
timeout -k 10 200 python3 -u tools/c_ab.py . base 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r5c1 seg8 1024 3 >> $L 2>&1 || exit 1
python3 tools/c_ab.py --compare base seg8 >> $L 2>&1
cat $L
timeout -k 10 400 python3 -u bench.py --config HB --batch 8 --steps 1 --warmup 0 > gpurun_out/prof_final/r05_bench_HB.json \
  2> gpurun_out/prof_final/r05_bench_HB.err
echo "HB rc=$?"
cat gpurun_out/prof_final/r05_bench_HB.json
