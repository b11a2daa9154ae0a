#!/bin/bash
# F1a with dW3 on MFMA (librlks.so) vs the DPP reduce-scatter (librlks_xp_base.so): phases at A = 2 / 4 / 8
# (8 keeps the DPP path), then the gradient parity tests
set -e
O=gpurun_out/${1:-r04h}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for a in 2; do
  for v in librlks_xp_base librlks librlks_xp_base librlks; do
    XP_A=$a RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_dw3.txt
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py tests/test_gpu_agent.py -k "grad or iteration or sgd" > $O/pytest_grad.log 2>&1 || { tail -40 $O/pytest_grad.log; exit 1; }
tail -3 $O/pytest_grad.log
