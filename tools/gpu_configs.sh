#!/bin/bash
# full GPU suite + smoke + bench lines for c2 / c3 / c4 (default) / c5 (one gpurun call)
set -e
O=gpurun_out/${1:-cfg}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 2 $O/pytest_gpu.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -n 1 $O/smoke.log
for c in c2 c3 c5; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.txt 2>&1
  tail -n 1 $O/bench_$c.txt | cut -c1-200
done
timeout -k 10 400 python3 -u bench.py > $O/bench_c4.txt 2>&1
tail -n 1 $O/bench_c4.txt | cut -c1-200
