# round 4: config E divergence diagnosis (per-QP traces GPU vs oracle), then the rest of the sco suite.
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
step gpurun_out/r4_g5_traceE.log timeout -k 10 300 python -u tools/trace_compare.py E 0 2
step gpurun_out/r4_g5_sco.log timeout -k 10 500 python -u -m pytest tests/test_gpu_sco.py -v --timeout 200 --timeout-method thread
