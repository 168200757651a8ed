# round 4: after reverting the a.x reuse -- torso_arm_8dof_C, bitwise against the previous build, E bench
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 200 python3 -u tools/torso_repeat.py . 2 > gpurun_out/r4_g35_torso.log 2>&1
timeout -k 10 300 python3 -u tools/build_bitwise.py . now > gpurun_out/r4_g35_now.log 2>&1
python3 tools/build_bitwise.py --compare prev now > gpurun_out/r4_g35_cmp.log 2>&1 || true
timeout -k 10 400 python3 -u bench.py --config E --batch 512 --inflight 3 --steps 3 --warmup 1 --no-cpu > gpurun_out/r04_bench_E.json 2> gpurun_out/bench_E.err
