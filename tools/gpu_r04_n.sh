#!/bin/bash
# F1a in 4-wave workgroups (librlks_xp_w4: workgroups drift out of phase, 3 per CU by LDS) vs 8-wave
set -e
O=gpurun_out/${1:-r04n}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for a in 2 8; do
for v in librlks librlks_xp_w4 librlks librlks_xp_w4; do
  XP_A=$a RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_w4.txt
done
done
RLKS_LIB=$L/librlks_xp_w4.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py -k "grad" > $O/pytest_w4.log 2>&1 || { tail -30 $O/pytest_w4.log; exit 1; }
tail -2 $O/pytest_w4.log
