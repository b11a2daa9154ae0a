#!/bin/bash
# round 6: node two-stream rollout + streamed policy head: parity tests, then same-box A/B bench lines
O=gpurun_out/r06b1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nodes.py tests/test_gpu_learn.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "node or wide" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
line() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 400 python3 -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), 'rollout_ms', round(k['rollout']['ms'],2), 'grad_ms', round(k['sgd_grad_total']['ms'],3))"
}
line c3_two c3 X=1 && line c3_one c3 RLKS_NODE_ONE_STREAM=1 && line c5_head c5 X=1 && line c5_gemm c5 RLKS_WIDE_HEAD_GEMM=1 && line c3_two_b c3 X=1 && line c3_one_b c3 RLKS_NODE_ONE_STREAM=1
