#!/bin/bash
# timing A/B of library variants (RLKS_LIB) on the bench's kernel timings; args: tag config variants...
set -e
O=gpurun_out/$1; C=$2; shift 2
mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then L=rl-k8s-scheduler_amd/rlks/librlks.so; else L=rl-k8s-scheduler_amd/rlks/librlks_xp_$v.so; fi
  RLKS_LIB=$L timeout -k 10 200 python3 -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $O/${C}_$v.txt 2>&1 || true
  python3 - $O/${C}_$v.txt <<'PY'
import json, sys
try:
    j = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
    k = j["kernels"]
    print(sys.argv[1], f"{j['value']/1e6:.2f}M", {n: round(k[n]["ms"] * 1000, 1) for n in ("k_sf_prep", "k_sf_fwd", "k_sf_bwd", "k_sf_dw2", "k_reduce", "sgd_grad_total") if n in k})
except Exception as e:
    print(sys.argv[1], "failed", open(sys.argv[1]).read()[-300:])
PY
done
