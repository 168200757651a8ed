#!/bin/bash
# Round 5 evidence on the final kernels: bench (config C) + rocprofv3 kernel
# stats + FETCH/WRITE passes (collect_profiles.sh), the phase profile of C,
# smoke(), and the host-loop bench line (config HB).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_final
(while sleep 45; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
bash tools/collect_profiles.sh r05 || exit 1
timeout -k 10 300 python3 -u tools/phase_profile.py C 1024 > gpurun_out/prof_final/r05_phase_profile_C.txt 2>&1 || exit 1
cp -n profiles/r05_* gpurun_out/prof_final/
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof_final/r05_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --config HB --batch 64 --steps 1 --warmup 1 > gpurun_out/prof_final/r05_bench_HB.json \
  2> gpurun_out/prof_final/r05_bench_HB.err
echo "HB rc=$?"
cat gpurun_out/bench.json gpurun_out/prof_final/r05_bench_HB.json
