#!/bin/bash
# A/B of SGD-step variant libraries (bench kernel table at c4) — RLKS_LIB picks the library
set -e
O=gpurun_out/ab_f2; mkdir -p $O
for L in "$@"; do
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/$L.txt 2>&1
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/$L.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$L', round(d['value']/1e6,3), {n:round(k[n]['ms']*1e3,1) for n in ('k_sf_fwd','k_sf_bwd','k_sf_dw2','k_reduce','k_sf_prep') if n in k})"
done
