#!/bin/bash
# A/B of the c3 node step across library builds (make OBJDIR=... OUT=... EXTRA=-D...): output
# lines under gpurun_out/$1/node_ab.txt
O=gpurun_out/${1:-iter}
mkdir -p $O
for L in librlks.so librlks_ab_lds.so librlks_ab_old.so; do
  [ -f rl-k8s-scheduler_amd/rlks/$L ] || continue
  echo "== $L" >> $O/node_ab.txt
  RLKS_LIB=rl-k8s-scheduler_amd/rlks/$L timeout -k 10 120 python3 tools/node_step_time.py >> $O/node_ab.txt 2>&1 || exit 1
done
cat $O/node_ab.txt
