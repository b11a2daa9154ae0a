#!/bin/bash
# Multi-rank rehearsal on one GPU (two ranks share it, gloo): the bench's barrier / max-over-ranks
# timing, the per-SGD-step gradient all-reduce and its instrumentation (the bench line's `allreduce`:
# allreduce_ms_per_sgd_step and its share of the iteration).  The 8-GPU RCCL run is the driver's.
set -e
O=gpurun_out/${1:-ranks}
mkdir -p $O
for C in c2 c4; do
  RLKS_DIST_BACKEND=gloo timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $C --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/bench_${C}_2ranks_gloo_1gpu.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/bench_${C}_2ranks_gloo_1gpu.log') if l.startswith('{')][-1]
print('$C', d['n_gpus'], round(d['value']/1e6,3), 'M', json.dumps(d['allreduce']))"
done
