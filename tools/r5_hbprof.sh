#!/bin/bash
# Round 5: rocprofv3 kernel trace + stats of the host-loop bench (config HB, 64 problems).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
rm -rf gpurun_out/prof_hb
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hb -o hb -- \
  python3 bench.py --config HB --batch 64 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_hb.log 2>&1
echo "rc=$?"
find gpurun_out/prof_hb -name "*stats*" | head
