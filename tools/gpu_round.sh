#!/bin/bash
# GPU test suite + smoke + default bench + rocprofv3 kernel stats of the bench (one gpurun call).
set -e
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 3 $O/pytest_gpu.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > $O/bench_c4.txt 2>&1
tail -n 1 $O/bench_c4.txt | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo done
