#!/bin/bash
# Round 6: phase profiles of config HA (B + JointAcc, waypoint-pair solve) and E
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/phase_profile.py HA 512 > gpurun_out/r6_pp_HA.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/phase_profile.py E 64 > gpurun_out/r6_pp_E.txt 2>&1 || exit 1
