#!/bin/bash
# round 6: k_sf_dw2r scheduling variants (F2R_SCHED builds, RLKS_LIB) against k_sf_dw2, same box
O=gpurun_out/r06_f2sched; mkdir -p $O
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
  line base_$r c4 X=1 && line s0_$r c4 RLKS_F2_REGS=1 && line s1_$r c4 RLKS_F2_REGS=1 RLKS_LIB=$L/librlks_xp_s1.so && \
  line s2_$r c4 RLKS_F2_REGS=1 RLKS_LIB=$L/librlks_xp_s2.so && line s3_$r c4 RLKS_F2_REGS=1 RLKS_LIB=$L/librlks_xp_s3.so || exit 1
done
