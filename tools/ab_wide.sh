#!/bin/bash
# A/B of variant libraries on the c5 wide-path gradient (tools/prof_wide.py): ab_wide.sh <lib>...
set -e
O=gpurun_out/ab_wide; mkdir -p $O
for L in "$@"; do
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 180 python3 -u tools/prof_wide.py --reps 6 > $O/$L.txt 2>&1
  echo "$L $(tail -1 $O/$L.txt)"
done
