#!/bin/bash
# A/B of variant libraries on one config's bench kernel table: ab_cfg.sh <config> <lib>...
set -e
C=$1; shift
O=gpurun_out/ab_cfg; mkdir -p $O
for L in "$@"; do
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 300 python3 -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $O/${C}_$L.txt 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/${C}_$L.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$C $L', round(d['value']/1e6,3), {n:round(k[n]['ms']*1e3,1) for n in ('k_sf_fwd','k_sf_bwd','k_sf_dw2','k_reduce','k_gather_packed') if n in k})"
done
