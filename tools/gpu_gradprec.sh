#!/bin/bash
# grad_precision.py over variant libraries (one process each): gpu_gradprec.sh <outdir> <lib>...
set -e
O=$1; shift
mkdir -p $O
for L in "$@"; do
  echo "== $L"
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 400 python3 -u tools/grad_precision.py --json $O/$L.json > $O/$L.txt 2>&1 || { tail -20 $O/$L.txt; exit 1; }
  grep -c "<" $O/$L.txt || true
done
