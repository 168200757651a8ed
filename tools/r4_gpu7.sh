# round 4: per-QP traces GPU vs oracle where the self-collision build parts (C continuous, C constraint, E).
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
step gpurun_out/r4_g7_Ccont.log timeout -k 10 300 python -u tools/trace_compare.py Ccont 0 3 8
step gpurun_out/r4_g7_Ccnt.log timeout -k 10 300 python -u tools/trace_compare.py Ccnt 0 1
step gpurun_out/r4_g7_E.log timeout -k 10 300 python -u tools/trace_compare.py E 0 2
