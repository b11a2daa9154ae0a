#!/bin/bash
# c3 node step: work-list kernel, chunk-total prefetch capped at 4 waves/SIMD (default) vs no prefetch
# vs prefetch uncapped (3 waves), and the lane-per-cluster kernel; parity of the default first
set -e
O=gpurun_out/${1:-r04v}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nodes.py > $O/nodes_suite.txt 2>&1 || { tail -40 $O/nodes_suite.txt; exit 1; }
tail -1 $O/nodes_suite.txt
for v in librlks librlks_xp_ec librlks librlks_xp_ec; do
  echo "== $v" | tee -a $O/node_wl.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_wl.txt
done
RLKS_LIB=$L/librlks_xp_CLOCK.so timeout -k 10 120 python3 -u tools/node_wl_clock.py 2>&1 | grep -v amdgpu.ids | tee $O/clock.txt
