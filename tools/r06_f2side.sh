#!/bin/bash
# round 6: F2 beside F1b on a side stream (RLKS_F2_SIDE=1) and F1a -> F2 -> F1b (=2) against the
# default order: gradient parity under each, then same-box alternating c4 bench lines
O=gpurun_out/r06_f2side; mkdir -p $O
for m in ${PYT:-}; do
  RLKS_F2_SIDE=$m timeout -k 10 400 python3 -u -m pytest tests/test_gpu_learn.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "ppo_grad_matches_oracle or fused_sgd_step or sgd_step_next or ppo_iteration" > $O/pytest_side$m.log 2>&1 || { tail -30 $O/pytest_side$m.log; exit 1; }
  tail -1 $O/pytest_side$m.log
done
line() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(k[n]['ms']*1e3,1) for n in ('k_sf_fwd','k_sf_bwd','k_sf_dw2','k_reduce','sgd_grad_total')}, {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
line base_a X=1 && line side_a RLKS_F2_SIDE=1 && line first_a RLKS_F2_SIDE=2 && \
line base_b X=1 && line side_b RLKS_F2_SIDE=1 && line first_b RLKS_F2_SIDE=2 && \
line base_c X=1 && line side_c RLKS_F2_SIDE=1 && line first_c RLKS_F2_SIDE=2
