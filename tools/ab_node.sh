#!/bin/bash
# A/B of the c3 node step across library builds (tools/build_variant.sh): ab_node.sh <lib>...
# output lines under gpurun_out/ab_node/node_ab.txt
set -e
O=gpurun_out/ab_node; mkdir -p $O
for L in "$@"; do
  echo "== $L" >> $O/node_ab.txt
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 120 python3 tools/node_step_time.py >> $O/node_ab.txt 2>&1
done
cat $O/node_ab.txt
