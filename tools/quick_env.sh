#!/bin/bash
# env-step / GAE parity tests + the default bench's kernel table (one gpurun call)
set -e
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_env.py tests/test_gpu_learn.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gae or vec_env or lean or gather or iteration or checkpoint or c4 or c1 or fused" > $O/pytest.log 2>&1
tail -n 2 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.txt 2>&1
tail -n 1 $O/bench.txt | cut -c1-300
