# Round-6 evidence of the generic-step build's workloads (run via gpurun):
# config HA bench line + rocprofv3 kernel stats, config E bench line
#   bash tools/gen_evidence.sh <round>
set -e
ROUND=${1:?round}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_final
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 400 python3 -u bench.py --config HA --batch 1024 --steps 6 --warmup 1 \
  > "profiles/${ROUND}_bench_HA.json" 2> gpurun_out/bench_HA.err
rm -rf gpurun_out/prof_ha
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ha -o ha -- \
  python3 bench.py --config HA --batch 1024 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_ha.log 2>&1
cp "$(find gpurun_out/prof_ha -name '*kernel_stats.csv' -print -quit)" "profiles/${ROUND}_kernel_stats_HA.csv"
timeout -k 10 600 python3 -u bench.py --config E --batch 512 --inflight 3 --steps 3 --warmup 1 --no-cpu \
  > "profiles/${ROUND}_bench_E.json" 2> gpurun_out/bench_E.err
cp profiles/${ROUND}_bench_HA.json profiles/${ROUND}_kernel_stats_HA.csv profiles/${ROUND}_bench_E.json gpurun_out/prof_final/
