#!/bin/bash
# round 6: F2 with H1 in registers (k_sf_dw2r, RLKS_F2_REGS=1) against k_sf_dw2: gradient parity under
# it, then same-box alternating c4 bench lines
O=gpurun_out/r06_f2regs; mkdir -p $O
RLKS_F2_REGS=1 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_learn.py tests/test_gpu_agent.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "ppo_grad_matches_oracle or sf16_grad or f16_throughput or fused_sgd_step or sgd_step_next or c4_shard or sf16_gradient_per_element" > $O/pytest_regs.log 2>&1 || { tail -40 $O/pytest_regs.log; exit 1; }
tail -1 $O/pytest_regs.log
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(k[n]['ms']*1e3,1) for n in ('k_sf_fwd','k_sf_bwd','k_sf_dw2','k_reduce','sgd_grad_total')}, {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
line base_a c4 X=1 && line regs_a c4 RLKS_F2_REGS=1 && line base_b c4 X=1 && line regs_b c4 RLKS_F2_REGS=1 && \
line c3_base c3 X=1 && line c3_regs c3 RLKS_F2_REGS=1
