set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 500 python3 -u bench.py --config E --batch 512 --inflight 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_E.json 2> gpurun_out/bench_E.err
