#!/bin/bash
# A/B of the W2 ring depth (librlks_xp_nb2.so: two buffers, the load of step st + 1 waited for at
# the end of step st; librlks.so: three where LDS allows): SGD phases at A = 2 / 8, then c4 bench
set -e
O=gpurun_out/${1:-r04f}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for a in 2 8; do
  for v in librlks_xp_nb2 librlks librlks_xp_nb2 librlks; do
    XP_A=$a RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/ab_ring.txt
  done
done
timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.txt 2>&1 || { tail -30 $O/bench_c4.txt; exit 1; }
RLKS_LIB=$L/librlks_xp_nb2.so timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4_nb2.txt 2>&1 || { tail -30 $O/bench_c4_nb2.txt; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("bench_c4", "bench_c4_nb2"):
    r = json.loads(open(f"{sys.argv[1]}/{f}.txt").read().strip().splitlines()[-1])
    k = r.get("kernels") or {}
    print(f, r["value"], r["ms_per_step"], {n: round(k[n]["ms"] * 1e3, 1) for n in ("k_sf_fwd", "k_sf_bwd", "k_sf_dw2", "sgd_grad_total", "rollout") if n in k})
PY
bash tools/profile_c3.sh > $O/profile_c3.txt 2>&1 || { tail -20 $O/profile_c3.txt; exit 1; }
tail -12 $O/profile_c3.txt
