#!/bin/bash
# round 6: LLVM AMDGPU scheduling strategies (whole library, -mllvm -amdgpu-sched-strategy=...) against
# the default build: gradient tests on each, then same-box c4 / c3 bench lines
L=$PWD/rl-k8s-scheduler_amd/rlks
O=gpurun_out/r06_sched; mkdir -p $O
for v in ilp mclause minreg; do
  RLKS_LIB=$L/librlks_xp_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_learn.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "ppo_grad_matches_oracle or fused_sgd_step" > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  echo $v $(tail -1 $O/pytest_$v.txt)
done
bash tools/r06_libab.sh sched c4 ilp mclause minreg && bash tools/r06_libab.sh sched c3 ilp mclause minreg
