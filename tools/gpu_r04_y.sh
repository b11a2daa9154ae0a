#!/bin/bash
# one-wave workgroups (W = 1) as the default: pairs per thread (NP 2 default, 1, 4), W = 4 and the
# lane-per-cluster kernel timed; then the GPU suite, smoke, c4 and c3 bench lines on the default
set -e
T=${1:-r04y}
O=gpurun_out/$T; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_np1 librlks_xp_np4 librlks_xp_w4 librlks_xp_ec librlks librlks_xp_np1 librlks_xp_np4; do
  echo "== $v" | tee -a $O/node_wl.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_wl.txt
done
bash tools/gpu_iter4.sh $T
timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3.txt 2>&1
tail -n 1 $O/bench_c3.txt | cut -c1-200
