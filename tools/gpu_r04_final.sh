#!/bin/bash
# end of round 4 on the final tree: node-step parity + times + phase clocks (tools/gpu_r04_v.sh), the
# evidence set (rocprofv3 of the bench, SGD PMC passes, GPU suite, smoke, c4 bench, suite against the
# debug library) and the c3 bench line
set -e
T=${1:-r04f}
bash tools/gpu_r04_v.sh $T
bash tools/gpu_r04_evidence.sh $T
timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/bench_c3.txt 2>&1
tail -n 1 gpurun_out/$T/bench_c3.txt | cut -c1-300
