#!/bin/bash
# round-4 iteration: F1a A/B (ws with global dZ2 stores vs old), node tests with the 16-row rollout
# forward, c3 / c4 bench lines
set -e
O=gpurun_out/${1:-r04b}; mkdir -p $O
bash tools/ab_f1a.sh old base noepi base 2>&1 | grep -v amdgpu.ids | tee $O/ab_f1a.txt
timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee $O/node_step.txt
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nodes.py > $O/pytest_nodes.log 2>&1 || { tail -40 $O/pytest_nodes.log; exit 1; }
tail -3 $O/pytest_nodes.log
timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.txt 2>&1 || { tail -30 $O/bench_c3.txt; exit 1; }
tail -2 $O/bench_c3.txt | cut -c1-1500
