#!/bin/bash
# round 6: same-box A/B of the working tree's F2 against the last commit's (librlks_xp_prev.so) and
# k_sf_dw2 (RLKS_F2_IMAGE=1), after the gradient tests on the working tree: r06_f2ab.sh <tag> [configs]
T=${1:-ab}; CF=${2:-c4}
O=gpurun_out/r06_f2ab_$T; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_learn.py tests/test_gpu_agent.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "ppo_grad_matches_oracle or sf16_grad or f16_throughput or fused_sgd_step or sgd_step_next or c4_shard or sf16_gradient_per_element" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
for c in $CF; do
  for r in a b; do
    line ${c}_new_$r $c X=1 && line ${c}_prev_$r $c RLKS_LIB=$L/librlks_xp_prev.so || exit 1
  done
  line ${c}_image $c RLKS_F2_IMAGE=1 || exit 1
done
