# the round's committed evidence on the final kernel (run via gpurun):
# latency model (micro benchmarks + phase profile), then bench + rocprofv3 kernel
# stats + FETCH/WRITE passes (collect_profiles.sh), copies into gpurun_out/prof_final/
set -e
ROUND=${1:-r03}
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python3 -u tools/latency_model.py "$ROUND" C 1024 > gpurun_out/latency.log 2>&1
bash tools/collect_profiles.sh "$ROUND"
mkdir -p gpurun_out/prof_final
timeout -k 10 200 python3 -u tools/phase_profile.py C 1024 > gpurun_out/prof_final/${ROUND}_phase_profile_C.txt 2>&1
cp -n profiles/${ROUND}_* gpurun_out/prof_final/
