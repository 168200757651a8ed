#!/bin/bash
# Round 6: phase profiles of config C (1024) on the shipped build and the
# -ffp-contract=off build (r6nc): where the contraction-off cycles go.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/r6_pp.log
: > $L
PP_ROOT=. timeout -k 10 200 python3 -u tools/phase_profile.py C 1024 > gpurun_out/r6_pp_base.txt 2>&1 || exit 1
PP_ROOT=r6nc timeout -k 10 200 python3 -u tools/phase_profile.py C 1024 > gpurun_out/r6_pp_nc.txt 2>&1 || exit 1
