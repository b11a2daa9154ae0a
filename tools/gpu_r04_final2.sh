#!/bin/bash
# the final tree (arrivals back in phase B): node-step parity + times + clocks, the GPU suite, smoke,
# c4 bench (tools/gpu_iter4.sh) and the c3 bench line
set -e
T=${1:-r04g}
bash tools/gpu_r04_v.sh $T
bash tools/gpu_iter4.sh $T
timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/bench_c3.txt 2>&1
tail -n 1 gpurun_out/$T/bench_c3.txt | cut -c1-200
