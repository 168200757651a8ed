# Round-6 evidence after the generic QP kernel's pass-scheduled forward solve and
# the generic-step build's d-value change (run via gpurun):
#   bash tools/hb_evidence.sh <round>
# config HB bench line (256 problems, cpu_baseline) + rocprofv3 stats of a
# 64-problem step; config HA bench line + rocprofv3 stats; config E bench line
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
timeout -k 10 400 python3 -u bench.py --config HA --batch 1024 --steps 6 --warmup 1 > $O/${ROUND}_bench_HA.json 2> gpurun_out/bench_HA.err
rm -rf gpurun_out/prof_ha
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ha -o ha -- \
  python3 bench.py --config HA --batch 1024 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_ha.log 2>&1
cp "$(find gpurun_out/prof_ha -name '*kernel_stats.csv' -print -quit)" $O/${ROUND}_kernel_stats_HA.csv
timeout -k 10 600 python3 -u bench.py --config E --batch 512 --inflight 3 --steps 3 --warmup 1 --no-cpu \
  > $O/${ROUND}_bench_E.json 2> gpurun_out/bench_E.err
