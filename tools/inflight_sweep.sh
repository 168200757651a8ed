# bench.py at the driver's step counts with 2, 3 and 4 batches in flight (no CPU baseline)
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
for n in 2 3 4; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu --inflight $n > gpurun_out/inflight_$n.json 2> gpurun_out/inflight_$n.err
done
