#!/bin/bash
# rocprofv3 evidence beyond the c2 headline (run on the GPU box from the repo root):
#   1. kernel trace + stats of bench.py --config c3 and --config c5 (one timed iteration each)
#   2. FETCH_SIZE / WRITE_SIZE passes (separate runs) over the node-step timing script, for the
#      HBM traffic of k_node_step (the step kernel of config c3)
# Outputs under gpurun_out/prof_<tag>/.  Every step has its own time limit; stop at the first failure.
set -e
TAG=${1:-cfg}
R=$(pwd)
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- \
  python3 $R/bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/c3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- \
  python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/c5.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/node_fetch -o p -- \
  python3 $R/tools/node_step_time.py > $O/node_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/node_write -o p -- \
  python3 $R/tools/node_step_time.py > $O/node_write.log 2>&1
echo profile_configs done
