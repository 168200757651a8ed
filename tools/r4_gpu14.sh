# round 4: after restoring the scene-contact row builder -- self pairs on/off parity (E wide, C continuous),
# the collision parity tests and E.
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
step gpurun_out/r4_g14_selfoff.log timeout -k 10 400 python -u tools/selfoff_parity.py
step gpurun_out/r4_g14_C.log timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v --timeout 300 --timeout-method thread -k "sqp_parity_collision or collision_rows or dual_arm_E"
