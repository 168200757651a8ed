# round 4: chunk sums loaded eight at a time, two hinge rows per thread -- bitwise check, E profile
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python3 -u tools/build_bitwise.py prevcmp prev > gpurun_out/r4_g30_prev.log 2>&1
timeout -k 10 300 python3 -u tools/build_bitwise.py . now > gpurun_out/r4_g30_now.log 2>&1
python3 tools/build_bitwise.py --compare prev now > gpurun_out/r4_g30_cmp.log 2>&1 || true
timeout -k 10 200 python3 -u tools/phase_profile.py E 512 > gpurun_out/r4_g30_phase_E.txt 2>&1
