#!/bin/bash
# end-of-session check of the committed tree: GPU suite + smoke + config benches (tools/gpu_configs.sh),
# then rocprofv3 kernel stats of the default (c4) bench
set -e
T=${1:-final}
bash tools/gpu_configs.sh $T
bash tools/prof_bench.sh $T
