#!/bin/bash
# Round 5: config C lone-batch A/B of two chain-solve variants against the main build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
L=gpurun_out/r5_c_ab2.log
: > $L
timeout -k 10 200 python3 -u tools/c_ab.py . base 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r5c1 nosched 1024 3 >> $L 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/c_ab.py r5c2 seg2 1024 3 >> $L 2>&1 || exit 1
python3 tools/c_ab.py --compare base nosched >> $L 2>&1
python3 tools/c_ab.py --compare base seg2 >> $L 2>&1
cat $L
