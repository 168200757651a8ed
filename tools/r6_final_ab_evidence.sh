# round 6, last GPU calls: the HB solve A/B, then the evidence lines (tools/hb_evidence.sh)
set -e
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
bash tools/hb_ab.sh 16
bash tools/hb_evidence.sh r06
