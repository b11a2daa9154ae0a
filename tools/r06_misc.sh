#!/bin/bash
# round 6 final tree: the fused F1 kernel (RLKS_F1_FUSED=1) against the two kernels again (no-SLP build,
# new F2), and the strong-scaling N = 1 anchor (1,048,576 lanes on one GPU)
O=gpurun_out/r06_misc; mkdir -p $O
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
line split_a c4 X=1 && line fused_a c4 RLKS_F1_FUSED=1 && line split_b c4 X=1 && line fused_b c4 RLKS_F1_FUSED=1 || exit 1
timeout -k 10 400 python3 -u bench.py --gpus 1 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline > $O/strong_n1.txt 2>&1 || { tail -5 $O/strong_n1.txt; exit 1; }
grep '^{' $O/strong_n1.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('strong N=1', round(d['value']/1e6,3), 'M', d['config'])"
