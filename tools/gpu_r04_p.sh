#!/bin/bash
# reduce kernel with batched partial loads (librlks.so) vs before (librlks_xp_base.so): SGD phases and
# the c4 bench's k_reduce, then the learner tests (bit-identity of fused / unfused and overlapped paths)
set -e
O=gpurun_out/${1:-r04p}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn.py tests/test_gpu_multirank.py > $O/pytest_red.log 2>&1 || { tail -40 $O/pytest_red.log; exit 1; }
tail -2 $O/pytest_red.log
for v in librlks_xp_base librlks librlks_xp_base librlks; do
  XP_A=2 RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_red.txt
done
for v in librlks_xp_base librlks; do
  RLKS_LIB=$L/$v.so timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.txt 2>&1 || { tail -20 $O/bench_$v.txt; exit 1; }
done
python3 - $O <<'PY'
import json, sys
for v in ("librlks_xp_base", "librlks"):
    r = json.loads(open(f"{sys.argv[1]}/bench_{v}.txt").read().strip().splitlines()[-1])
    k = r["kernels"]
    print(v, round(r["value"] / 1e6, 3), {n: round(k[n]["ms"] * 1e3, 1) for n in ("k_reduce", "sgd_grad_total", "k_sf_fwd") if n in k})
PY
