# round 4: the round-3 build and the current one on config C continuous, same box.
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
step gpurun_out/r4_g10_r3.log timeout -k 10 300 python -u tools/r3_ccont.py "$PWD/r3cmp"
step gpurun_out/r4_g10_now.log timeout -k 10 300 python -u tools/r3_ccont.py "$PWD"
