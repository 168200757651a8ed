# round 4: C constraint parity with the grown cloud, jitter gaps, drop-in, sco, then the bench line.
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
step gpurun_out/r4_g15_C.log timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v -s --timeout 300 --timeout-method thread -k "collision_constraint or jitter"
step gpurun_out/r4_g15_dropin.log timeout -k 10 500 python -u -m pytest tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread
step gpurun_out/r4_g15_sco.log timeout -k 10 300 python -u -m pytest tests/test_gpu_sco.py -v --timeout 200 --timeout-method thread -k batched
