#!/bin/bash
# round-4 probe: F1a variants A/B + their SQ / icache counters, the c3 node-step timing and its
# rocprofv3 anatomy (tools/profile_c3.sh)
set -e
O=gpurun_out/${1:-r04probe}; mkdir -p $O
bash tools/ab_f1a.sh old base noepi all3 base 2>&1 | grep -v amdgpu.ids | tee $O/ab_f1a.txt
bash tools/pmc_f1a.sh ${1:-r04probe}/pmc_f1a base old 2>&1 | grep -v amdgpu.ids | tee $O/pmc_f1a.txt
timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee $O/node_step.txt
