# round 4: drop-in + host-loop batching + stream + planning EXPECTs, then the bench line.
# A pytest step that only had test failures (exit 1) lets the next step run; a time
# limit, abort or crash (any other nonzero status) ends the script there.
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
step gpurun_out/r4_g3_dropin.log timeout -k 10 1000 python -u -m pytest tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread
step gpurun_out/r4_g3_batched.log timeout -k 10 900 python -u -m pytest tests/test_gpu_sco.py -v --timeout 300 --timeout-method thread -k batched
step gpurun_out/r4_g3_front.log timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v --timeout 300 --timeout-method thread -k "frontdoor_single or dynamic_problem_assignment or stream_batches or reference_planning"
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
