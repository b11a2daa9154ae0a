#!/bin/bash
# fused F1 (k_sf_f1) vs the two kernels (RLKS_F1_SPLIT=1) on one box: the gradient tests on the fused
# kernel, then c4 / c3 bench lines of both
set -e
O=gpurun_out/f1fused; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_learn.py tests/test_gpu_agent.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ppo_grad_matches or sf16_grad or tile_dynamic or fused_sgd or step_next or c4_shard or f16_throughput or iteration_matches" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c4 c3; do
  for v in split fused split fused; do
    if [ $v = split ]; then export RLKS_F1_SPLIT=1; else unset RLKS_F1_SPLIT; fi
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > $O/${cfg}_$v.txt 2>&1
    python3 -c "
import json
d=[json.loads(l) for l in open('$O/${cfg}_$v.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$cfg $v', round(d['value']/1e6,3), {n:round(k[n]['ms']*1e3,1) for n in ('k_sf_fwd','k_sf_bwd','f1_total','k_sf_dw2','k_reduce','sgd_grad_total') if n in k})"
  done
done
