#!/bin/bash
# round 6: the library built with -fno-slp-vectorize (no packed-f32 VALU beside the MFMAs) against the
# default build: gradient tests on it, then same-box c4 / c3 bench lines
L=$PWD/rl-k8s-scheduler_amd/rlks
O=gpurun_out/r06_libab_noslp; mkdir -p $O
RLKS_LIB=$L/librlks_xp_noslp.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_learn.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "ppo_grad_matches_oracle or fused_sgd_step or sgd_step_next" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/r06_libab.sh noslp c4 noslp && bash tools/r06_libab.sh noslp c3 noslp
