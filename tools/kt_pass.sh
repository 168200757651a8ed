# the rocprofv3 kernel-trace pass alone, at the driver's step counts (tools/collect_profiles.sh step 2)
set -e
export TMPDIR=/tmp
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
rm -rf gpurun_out/prof_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_kt.log 2>&1
