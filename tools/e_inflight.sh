# config E bench (512 problems) with three batches in flight, for comparison with tools/e_bench.sh's two
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python3 -u bench.py --config E --batch 512 --inflight ${1:-3} --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_E${1:-3}.json 2> gpurun_out/bench_E${1:-3}.err
