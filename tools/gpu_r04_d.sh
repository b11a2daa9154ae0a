#!/bin/bash
# c2 rollout A/B (persistent k_sf_roll vs per-step k_sf_fwd16 + k_sample_step), then the full GPU
# suite + smoke + c4 bench (tools/gpu_iter4.sh)
O=gpurun_out/${1:-r04d}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 300 python3 -u bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c2.txt 2>&1 || { tail -30 $O/bench_c2.txt; exit 1; }
RLKS_LIB=$L/librlks_xp_step.so timeout -k 10 300 python3 -u bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c2_step.txt 2>&1 || { tail -30 $O/bench_c2_step.txt; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("bench_c2", "bench_c2_step"):
    r = json.loads(open(f"{sys.argv[1]}/{f}.txt").read().strip().splitlines()[-1])
    k = r.get("kernels") or {}
    print(f, r["value"], r["ms_per_step"], json.dumps(k.get("rollout")))
PY
bash tools/gpu_iter4.sh ${1:-r04d}
