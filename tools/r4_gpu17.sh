# round 4: jitter gaps (element-wise QP steps), C constraint parity with the 49-run cloud, user cost, batched host loops.
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
step gpurun_out/r4_g17_C.log timeout -k 10 500 python -u -m pytest tests/test_gpu.py -v -s --timeout 400 --timeout-method thread -k "collision_constraint or jitter"
step gpurun_out/r4_g17_sco.log timeout -k 10 300 python -u -m pytest tests/test_gpu_sco.py -v --timeout 200 --timeout-method thread -k "batched and fixed"
