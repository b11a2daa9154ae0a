#!/bin/bash
# per-wave phase clocks of the c3 work-list node step
set -e
O=gpurun_out/${1:-r04w}; mkdir -p $O
RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/librlks_xp_CLOCK.so timeout -k 10 120 python3 -u tools/node_wl_clock.py 2>&1 | grep -v amdgpu.ids | tee $O/clock.txt
