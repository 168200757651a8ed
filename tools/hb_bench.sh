# config HB bench line (256 problems, cpu_baseline) + rocprofv3 stats of a 64-problem step (run via gpurun)
#   bash tools/hb_bench.sh <round>
set -e
ROUND=${1:?round}
export TMPDIR=/tmp
O=gpurun_out/prof_final
mkdir -p $O
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 400 python3 -u bench.py --config HB --batch 256 --steps 1 --warmup 0 > $O/${ROUND}_bench_HB.json 2> gpurun_out/bench_HB.err
rm -rf gpurun_out/prof_hb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hb -o hb -- \
  python3 bench.py --config HB --batch 64 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_hb.log 2>&1
cp "$(find gpurun_out/prof_hb -name '*kernel_stats.csv' -print -quit)" $O/${ROUND}_kernel_stats_HB.csv
