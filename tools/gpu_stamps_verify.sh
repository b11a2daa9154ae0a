#!/bin/bash
# F1a phase stamps (diagnostic library), then the full GPU suite + smoke + config benches
set -e
O=gpurun_out/${1:-r02d}
mkdir -p $O
RLKS_LIB=rl-k8s-scheduler_amd/rlks/librlks_stamps.so timeout -k 10 180 python3 -u tools/stamps.py > $O/stamps_fwd.txt 2>&1
cat $O/stamps_fwd.txt
bash tools/gpu_configs.sh ${1:-r02d}
