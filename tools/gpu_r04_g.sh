#!/bin/bash
# c3 node-step occupancy A/B: k_node_step_ec held to 6 / 8 waves per SIMD (spills) vs the default (97 VGPRs, 4)
set -e
O=gpurun_out/${1:-r04g}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_wpe6 librlks_xp_wpe8 librlks librlks_xp_wpe6 librlks_xp_wpe8; do
  echo "== $v" | tee -a $O/node_ab.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_ab.txt
done
