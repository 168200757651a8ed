# round 4: the sparse-LDL generic QP (sco surface), self-collision rows + config E parity, then the bench line.
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
step gpurun_out/r4_g4_sco.log timeout -k 10 500 python -u -m pytest tests/test_gpu_sco.py -x -v --timeout 200 --timeout-method thread
step gpurun_out/r4_g4_self.log timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v --timeout 250 --timeout-method thread -k "collision_rows or dual_arm"
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
