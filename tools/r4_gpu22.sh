# round 4: counter passes for config C and E, E bench (inflight 3) and phase profile, arm_6dof_A parity record
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
bash tools/pmc_latency.sh r04 C 1024 > gpurun_out/pmc_C.log 2>&1
timeout -k 10 400 python3 -u bench.py --config E --batch 512 --inflight 3 --steps 3 --warmup 1 --no-cpu > gpurun_out/r04_bench_E.json 2> gpurun_out/bench_E.err
timeout -k 10 200 python3 -u tools/phase_profile.py E 512 > gpurun_out/r04_phase_profile_E.txt 2>&1
bash tools/pmc_latency.sh r04 E 512 > gpurun_out/pmc_E.log 2>&1
mkdir -p gpurun_out/prof_final
cp profiles/r04_pmc_* gpurun_out/prof_final/
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -k "arm_6dof_A" > gpurun_out/r4_g22.log 2>&1 || true
cp gpurun_out/parity_table.json gpurun_out/r4_parity_table_g22.json
