#!/bin/bash
# librlks_xp_<name>.so: the whole working-tree library built with extra hipcc flags into its own
# object directory, for same-box A/B runs (RLKS_LIB=... ; tools/ab_cfg.sh, tools/grad_precision.py):
#   build_variant.sh <name> [hipcc flags...]      (no flags: the tree as it stands)
set -e
N=$1; shift
C="$(cd "$(dirname "$0")/../rl-k8s-scheduler_amd/csrc" && pwd)"
make -s -C "$C" -j8 OUT=../rlks/librlks_xp_$N.so OBJDIR=../build/xp_$N EXTRA="$*" ../rlks/librlks_xp_$N.so
