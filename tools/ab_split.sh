#!/bin/bash
# A/B of the fused F1 kernel vs the split F1a/F1b pair over the BASELINE configs (bench kernel timing).
set -e
O=gpurun_out/ab_split
mkdir -p $O
for c in c2 c3 c4; do
  for s in 0 1; do
    RLKS_F1_SPLIT=$s timeout -k 10 240 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/${c}_s$s.log 2>&1
    tail -n 1 $O/${c}_s$s.log
  done
done
