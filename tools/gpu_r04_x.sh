#!/bin/bash
# c3 node step: waves per workgroup of k_node_step_wl (4 = default, 2, 1): parity of each + times
set -e
O=gpurun_out/${1:-r04x}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_w2 librlks_xp_w1; do
  RLKS_LIB=$L/$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nodes.py > $O/nodes_suite_$v.txt 2>&1 || { tail -30 $O/nodes_suite_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/nodes_suite_$v.txt)"
done
for v in librlks librlks_xp_w2 librlks_xp_w1 librlks_xp_ec librlks librlks_xp_w2 librlks_xp_w1; do
  echo "== $v" | tee -a $O/node_wl.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_wl.txt
done
