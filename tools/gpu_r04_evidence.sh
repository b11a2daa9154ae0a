#!/bin/bash
# round-4 evidence on the committed tree: rocprofv3 of the bench command + SGD PMC passes
# (tools/profile_round.sh), the GPU suite + smoke + c4 bench (tools/gpu_iter4.sh), the suite against
# the bounds-checked debug library
set -e
T=${1:-r04}
bash tools/profile_round.sh $T
bash tools/gpu_iter4.sh $T
O=gpurun_out/$T
RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/librlks_debug.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu_debug.log 2>&1 || true
tail -3 $O/pytest_gpu_debug.log
