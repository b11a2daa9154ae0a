#!/bin/bash
# F1a with both nets a wave (k_sf_fwd2, librlks.so) vs the 16-row kernel (librlks_xp_base.so), A = 2 / 4,
# then the SGD-step parity tests on the new kernel
set -e
O=gpurun_out/${1:-r04o}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py -k "grad or dynamic" > $O/pytest_fw2.log 2>&1 || { tail -40 $O/pytest_fw2.log; exit 1; }
tail -2 $O/pytest_fw2.log
for a in 2 4; do
for v in librlks_xp_base librlks librlks_xp_base librlks; do
  XP_A=$a RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_fw2.txt
done
done
