#!/bin/bash
# same-box A/B of SGD-step phase timings over the librlks_xp_*.so variants named on the command line
for v in "$@"; do
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/librlks_xp_$v.so timeout -k 10 120 python3 -u tools/xp_f1a_time.py || exit 1
done
