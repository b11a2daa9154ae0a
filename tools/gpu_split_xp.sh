#!/bin/bash
# GPU learn/agent tests on the current library, then split-kernel A/B against HEAD's sgd_sf16.hip
set -e
O=gpurun_out/split_xp; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_learn.py tests/test_gpu_agent.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/xp_f1a.sh split_xp c4 base head base head
