#!/bin/bash
# Round 5: a.x-reuse traces (HEAD / reuse / probe builds) and the per-pair collision GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 100 python -u tools/ax_trace.py . head > gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 100 python -u tools/ax_trace.py r5ax2 reuse >> gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 100 python -u tools/ax_trace.py r5ax probe >> gpurun_out/r5_axtrace.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "pairs" > gpurun_out/r5_pairs.log 2>&1
echo "rc=$?"
tail -5 gpurun_out/r5_axtrace.log; tail -15 gpurun_out/r5_pairs.log
