#!/bin/bash
# round 6 final tree: the other BASELINE configs' bench lines (c2, c3, c5) and a two-rank launcher run
# (gloo, both ranks on the one GPU), same box
O=gpurun_out/r06_cfgs; mkdir -p $O
for c in c2 c3 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$c.txt 2>&1 || { tail -10 $O/bench_$c.txt; exit 1; }
  grep '^{' $O/bench_$c.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print('$c', round(d['value']/1e6,3), 'M env-steps/s, ms/it', round(d['ms_per_step'],1), r.get('kernel'), round(r.get('frac',0),3))"
done
RLKS_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4_gpus2_gloo.txt 2>&1 || { tail -10 $O/bench_c4_gpus2_gloo.txt; exit 1; }
grep '^{' $O/bench_c4_gpus2_gloo.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('c4 --gpus 2 (gloo, one GPU)', round(d['value']/1e6,3), 'M, n_gpus', d['n_gpus'], 'allreduce', d.get('allreduce'))"
