#!/bin/bash
# The round's committed evidence on the final kernel (run on the GPU box via gpurun):
#   bash tools/round_evidence.sh <round>
#   1. serial-floor model of config C       -> profiles/<round>_latency_C.json (tools/latency_model.py)
#   2. counter passes of one lone C batch    -> profiles/<round>_pmc_C.json (tools/pmc_latency.sh)
#   3. bench line + rocprofv3 kernel stats + FETCH/WRITE passes (tools/collect_profiles.sh)
#                                            -> profiles/<round>_{bench,kernel_stats,pmc_hbm}.*
#   4. phase profile of C                    -> profiles/<round>_phase_profile_C.txt
#   5. config HA (B + JointAcc, waypoint-pair solve): bench line and rocprofv3 kernel stats
#                                            -> profiles/<round>_bench_HA.json, <round>_kernel_stats_HA.csv
# Every step has its own time limit; the first failure ends the script. The
# new profiles are copied to gpurun_out/prof_final/ (what gpurun brings back).
set -e
ROUND=${1:?round, e.g. r06}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_final
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python3 -u tools/latency_model.py "$ROUND" C 1024 > gpurun_out/latency.log 2>&1
bash tools/pmc_latency.sh "$ROUND" C 1024 > gpurun_out/pmc_C.log 2>&1
bash tools/collect_profiles.sh "$ROUND"
timeout -k 10 300 python3 -u tools/phase_profile.py C 1024 > "profiles/${ROUND}_phase_profile_C.txt" 2>&1
timeout -k 10 400 python3 -u bench.py --config HA --batch 1024 --steps 6 --warmup 1 \
  > "profiles/${ROUND}_bench_HA.json" 2> gpurun_out/bench_HA.err
rm -rf gpurun_out/prof_ha
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ha -o ha -- \
  python3 bench.py --config HA --batch 1024 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_ha.log 2>&1
cp "$(find gpurun_out/prof_ha -name '*kernel_stats.csv' -print -quit)" "profiles/${ROUND}_kernel_stats_HA.csv"
cp profiles/${ROUND}_* gpurun_out/prof_final/
