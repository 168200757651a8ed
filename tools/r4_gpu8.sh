# round 4: fused-kernel contact rows vs the oracle along init -> solution paths (C continuous, C, E).
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
step gpurun_out/r4_g8_Ccont.log timeout -k 10 300 python -u tools/rows_sweep.py Ccont 16 200 21
step gpurun_out/r4_g8_E.log timeout -k 10 300 python -u tools/rows_sweep.py E 4 0 11
step gpurun_out/r4_g8_selfoff.log timeout -k 10 400 python -u tools/selfoff_parity.py
