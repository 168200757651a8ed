# round 4: batches in flight sweep for config C
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
for k in 2 4 6; do
  timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu --inflight $k > gpurun_out/r4_g28_if$k.json 2> gpurun_out/r4_g28_if$k.err
done
