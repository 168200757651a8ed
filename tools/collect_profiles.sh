#!/bin/bash
# Collect the round's committed profiles on the GPU box (run via gpurun):
#   1. bench.py (default config, with cpu_baseline)       -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench  -> gpurun_out/prof_kt/
#   3. rocprofv3 --pmc FETCH_SIZE (own pass)               -> gpurun_out/prof_fetch/
#   4. rocprofv3 --pmc WRITE_SIZE (own pass)               -> gpurun_out/prof_write/
# then tools/summarize_profiles.py writes profiles/<round>_*.
set -e
ROUND=${1:-r01}
export TMPDIR=/tmp
rm -rf gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_write.log 2>&1
python3 tools/summarize_profiles.py "$ROUND"
