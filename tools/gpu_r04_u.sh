#!/bin/bash
# SQ anatomy of the c3 node step: work-list kernel with / without the chunk-total prefetch, and the
# lane-per-cluster kernel
set -e
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_NOPF librlks_xp_ec; do
  RLKS_LIB=$L/$v.so bash tools/pmc_any.sh ${1:-r04u}_$v tools/node_step_time.py
  python3 tools/pmc_anatomy.py gpurun_out/${1:-r04u}_$v k_node_step > /dev/null
  rm -rf gpurun_out/${1:-r04u}_$v/{a,b,trace}
  cat gpurun_out/${1:-r04u}_$v/summary.txt
done
