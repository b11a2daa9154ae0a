#!/bin/bash
# same-box A/B of the default library against variant libraries: r06_libab.sh <tag> <config> <lib>...
T=$1; CF=$2; shift 2
O=gpurun_out/r06_libab_$T; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
for r in a b; do
  line ${CF}_base_$r $CF X=1 || exit 1
  for v in "$@"; do line ${CF}_${v}_$r $CF RLKS_LIB=$L/librlks_xp_$v.so || exit 1; done
done
