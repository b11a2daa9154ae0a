#!/bin/bash
# librlks_xp_head.so: the library as committed (HEAD, or the commit given), built from a scratch
# worktree, for same-box A/B timing against the working tree (tools/ab_cfg.sh)
set -e
REF=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/rlks_head_wt
rm -rf $T && git -C $R worktree prune && git -C $R worktree add --detach $T $REF > /dev/null
make -C $T/rl-k8s-scheduler_amd/csrc -j8 OUT=$R/rl-k8s-scheduler_amd/rlks/librlks_xp_head.so OBJDIR=/tmp/rlks_head_obj > /dev/null
git -C $R worktree remove --force $T
