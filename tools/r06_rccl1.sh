#!/bin/bash
# RCCL on one GPU: the multi-rank SGD step with a one-rank RCCL process group (RLKS_DDP_FORCE=1): the
# multirank GPU tests (incl. parameters bit-identical to the one-rank path) and a c4 bench line
O=gpurun_out/r06_rccl1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -s -k one_rank_rccl --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED|one-rank RCCL" $O/pytest.log | cut -c1-400
RLKS_DDP_FORCE=1 timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_forced.txt 2>&1 || { tail -20 $O/bench_forced.txt; exit 1; }
grep '^{' $O/bench_forced.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('forced one-rank RCCL c4', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],1), 'ms/it', json.dumps(d['allreduce']))"
