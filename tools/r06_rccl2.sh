#!/bin/bash
# the multi-rank SGD step's host cost on one GPU (one-rank RCCL group, RLKS_DDP_FORCE=1): c4 bench lines
# with the overlapped two-bucket all-reduce and with one bucket, beside the ordinary one-rank line;
# plus a host-side profile of the per-step Python calls
O=gpurun_out/r06_rccl2; mkdir -p $O
line() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/$n.txt 2>&1 || { tail -20 $O/$n.txt; return 1; }
  grep '^{' $O/$n.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); a=d.get('allreduce') or {}
print('$n', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],1), 'ms/it', 'exposed_ms/step', a.get('allreduce_ms_per_sgd_step'))"
}
line one_rank X=1 && line forced_overlap RLKS_DDP_FORCE=1 && line forced_onebucket RLKS_DDP_FORCE=1 RLKS_OVERLAP_ALLREDUCE=0 || exit 1
RLKS_DDP_FORCE=1 timeout -k 10 300 python3 -u tools/host_step_cost.py > $O/host_cost.txt 2>&1; cat $O/host_cost.txt | tail -25
