#!/bin/bash
# reduce partial-load batching: 8 (librlks.so) vs 4 (librlks_xp_rb4) vs none (librlks_xp_base), c4 bench k_reduce
set -e
O=gpurun_out/${1:-r04q}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks_xp_base librlks_xp_rb4 librlks librlks_xp_rb4 librlks; do
  RLKS_LIB=$L/$v.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$v.txt 2>&1 || { tail -20 $O/bench_$v.txt; exit 1; }
  python3 - $O/bench_$v.txt $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = r["kernels"]
print(sys.argv[2], round(r["value"] / 1e6, 3), {n: round(k[n]["ms"] * 1e3, 1) for n in ("k_reduce", "sgd_grad_total") if n in k})
PY
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py -k "fused or grad or iteration" > $O/pytest_rb8.log 2>&1 || { tail -30 $O/pytest_rb8.log; exit 1; }
tail -2 $O/pytest_rb8.log
