# round 4 final kernel: bench + rocprofv3 stats + FETCH/WRITE + latency model + phase profiles C and E
set -e
bash tools/final_evidence.sh r04
timeout -k 10 200 python3 -u tools/phase_profile.py E 512 > gpurun_out/prof_final/r04_phase_profile_E.txt 2>&1
