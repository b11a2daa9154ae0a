#!/bin/bash
# GPU learn / agent / multi-rank tests (the next-minibatch gather chained on both step forms)
set -e
O=gpurun_out/chain_ranks; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_learn.py tests/test_gpu_agent.py tests/test_gpu_multirank.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
