set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
bash tools/pmc_latency.sh r03 E 512 > gpurun_out/pmc_E.log 2>&1
