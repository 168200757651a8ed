# round 4: counter passes, config C then config E (separate logs)
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
bash tools/pmc_latency.sh r04 C 1024 > gpurun_out/pmc_C.log 2>&1
mkdir -p gpurun_out/prof_final
cp profiles/r04_pmc_C.json gpurun_out/prof_final/
bash tools/pmc_latency.sh r04 E 512 > gpurun_out/pmc_E.log 2>&1
cp profiles/r04_pmc_E.json gpurun_out/prof_final/
