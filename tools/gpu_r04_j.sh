#!/bin/bash
# F1a main-loop A/B: one barrier per k-tile with both W2 n-halves per step (librlks_xp_big) vs two,
# with and without the epilogue (the noepi builds are timing ablations), A = 2; then the big
# build's gradient parity
set -e
O=gpurun_out/${1:-r04j}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_big librlks_xp_noepi librlks_xp_bignoepi librlks librlks_xp_big librlks_xp_noepi librlks_xp_bignoepi; do
  XP_A=2 RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_big.txt
done
RLKS_LIB=$L/librlks_xp_big.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py -k "grad" > $O/pytest_big.log 2>&1 || { tail -30 $O/pytest_big.log; exit 1; }
tail -2 $O/pytest_big.log
