#!/bin/bash
# one GPU iteration on the current tree: the -m gpu suite (all failures reported), smoke, then the
# default (c4) bench (only if the suite passed); logs under gpurun_out/$1
O=gpurun_out/${1:-iter}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?
tail -25 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (reported above); anything else: stop
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
python3 - $O/bench.txt <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=r["kernels"]
print("value %.3fM env-steps/s  ms/iter %.1f" % (r["value"]/1e6, r["ms_per_step"]))
for n in ("k_sf_prep","k_sf_fwd","k_sf_bwd","f1_total","k_sf_dw2","k_reduce","sgd_grad_total","rollout","k_gae"):
    if n in k: print(n, round(k[n]["ms"]*1e3,1), "us", round(k[n].get("frac_sf16_mfma",0),3))
PY
