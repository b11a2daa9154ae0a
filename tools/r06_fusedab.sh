#!/bin/bash
# round 6 final tree: fused F1 (RLKS_F1_FUSED=1) against the two kernels, three alternations at c4, two
# at c3 and c2
O=gpurun_out/r06_fusedab; mkdir -p $O
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1))"
}
for r in a b c; do line c4_split_$r c4 X=1 && line c4_fused_$r c4 RLKS_F1_FUSED=1 || exit 1; done
for r in a b; do line c3_split_$r c3 X=1 && line c3_fused_$r c3 RLKS_F1_FUSED=1 || exit 1; done
for r in a b; do line c2_split_$r c2 X=1 && line c2_fused_$r c2 RLKS_F1_FUSED=1 || exit 1; done
