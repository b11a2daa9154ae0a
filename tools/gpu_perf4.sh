#!/bin/bash
# perf check of the current tree without the test suite: optional micro test, then the c4 bench's
# kernel table; logs under gpurun_out/$1
O=gpurun_out/${1:-perf}
mkdir -p $O
if [ -x tools/micro/mfma_round ]; then timeout -k 10 120 ./tools/micro/mfma_round > $O/mfma_round.txt 2>&1 && cat $O/mfma_round.txt; fi
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
python3 - $O/bench.txt <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=r["kernels"]
print("value %.3fM env-steps/s  ms/iter %.1f" % (r["value"]/1e6, r["ms_per_step"]))
for n in ("k_sf_prep","k_sf_fwd","k_sf_bwd","f1_total","k_sf_dw2","k_reduce","sgd_grad_total","rollout","k_gae"):
    if n in k: print(n, round(k[n]["ms"]*1e3,1), "us", round(k[n].get("frac_sf16_mfma",0),3))
PY
