set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python -u bench.py > gpurun_out/r4_base_bench.json 2> gpurun_out/r4_base_bench.err
timeout -k 10 200 python -u tools/phase_profile.py C 1024 > gpurun_out/r4_base_phaseC.txt 2>&1
timeout -k 10 300 python -u tools/phase_profile.py E 64 > gpurun_out/r4_base_phaseE.txt 2>&1
