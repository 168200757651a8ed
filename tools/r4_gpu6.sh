# round 4: self-collision (hit-bit sizing fix) + config E parity, the jitter-gap measurement, the C parity and bench.
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
step() {
  log=$1
  shift
  "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step failed with $rc: $*" >> gpurun_out/r4_steps.log; exit $rc; fi
}
step gpurun_out/r4_g6_self.log timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v -s --timeout 250 --timeout-method thread -k "collision_rows_parity_self or dual_arm_E or jitter"
step gpurun_out/r4_g6_C.log timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v --timeout 250 --timeout-method thread -k "sqp_parity_collision or collision_rows_parity"
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench6.json 2> gpurun_out/r4_bench6.err
