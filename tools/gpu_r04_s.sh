#!/bin/bash
# c3 node step: work-list kernel (librlks, default) parity + time vs the lane-per-cluster kernel (librlks_xp_ec)
set -e
O=gpurun_out/${1:-r04s}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nodes.py > $O/nodes_suite.txt 2>&1 || { tail -40 $O/nodes_suite.txt; exit 1; }
tail -3 $O/nodes_suite.txt
for v in librlks librlks_xp_ec librlks_xp_np1 librlks_xp_np4 librlks librlks_xp_ec librlks_xp_np4; do
  echo "== $v" | tee -a $O/node_wl.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_wl.txt
done
