# round 4: per-QP traces of the C-1024 / D-rank7 problems outside the cloud envelope
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
for p in 209 331 613 8005; do
  timeout -k 10 200 python -u tools/trace_compare.py C@$p 0 > gpurun_out/r4_g19_$p.log 2>&1 || exit $?
done
