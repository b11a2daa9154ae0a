#!/bin/bash
# timing only: the c4 SGD-step kernels with the two F1 kernels (default), the fused F1 (RLKS_F1_FUSED=1)
# and the given variant libraries, one box
O=gpurun_out/f1time; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; p=k.get('pipeline',{}).get('ms',{})
print('$n', round(d['value']/1e6,3), 'grad', round(k['sgd_grad_total']['ms']*1e3,1), 'pipeline', {a:round(b*1e3,1) for a,b in p.items()})"
}
for i in 1 2 3; do
  run split RLKS_X=0 && run fused RLKS_F1_FUSED=1 || exit 1
  for L in "$@"; do run $L RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L || exit 1; done
done
