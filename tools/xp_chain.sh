#!/bin/bash
# A/B: next-minibatch gather inside the reduce launch (chain) vs separate gather launches
O=gpurun_out/xp_chain; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_learn.py tests/test_gpu_agent.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in chain nochain; do
    if [ $v = nochain ]; then export RLKS_XP_NOCHAIN=1; else unset RLKS_XP_NOCHAIN; fi
    timeout -k 10 200 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_${v}_$r.txt 2>&1 || exit 1
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[1], round(j['value']/1e6,3), j['ms_per_step'])" $O/c4_${v}_$r.txt
  done
done
