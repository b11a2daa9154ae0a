#!/bin/bash
# round-4 iteration: F1a A/B (ws with global dZ2 stores vs old), node tests with the 16-row rollout
# forward, c3 bench, c4 rollout A/B (fused k_sf_roll vs per-step k_sf_fwd16 + k_sample_step)
set -e
O=gpurun_out/${1:-r04b}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
bash tools/ab_f1a.sh old base noepi base 2>&1 | grep -v amdgpu.ids | tee $O/ab_f1a.txt
timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee $O/node_step.txt
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nodes.py > $O/pytest_nodes.log 2>&1 || { tail -40 $O/pytest_nodes.log; exit 1; }
tail -3 $O/pytest_nodes.log
timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3.txt 2>&1 || { tail -30 $O/bench_c3.txt; exit 1; }
tail -1 $O/bench_c3.txt | cut -c1-1500
timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.txt 2>&1 || { tail -30 $O/bench_c4.txt; exit 1; }
RLKS_LIB=$L/librlks_xp_step.so timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4_step.txt 2>&1 || { tail -30 $O/bench_c4_step.txt; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("bench_c3", "bench_c4", "bench_c4_step"):
    r = json.loads(open(f"{sys.argv[1]}/{f}.txt").read().strip().splitlines()[-1])
    k = r.get("kernels") or {}
    print(f, r["value"], r["ms_per_step"], json.dumps({n: k[n] for n in ("rollout", "k_node_step_c3", "k_sf_fwd", "sgd_grad_total") if n in k})[:900])
PY
