#!/bin/bash
# Round 6: per-QP traces of the JointAcc parity misses (B-acc problems 1, 26)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/trace_compare.py B-acc 1 26 > gpurun_out/r6_jacc_trace.log 2>&1
