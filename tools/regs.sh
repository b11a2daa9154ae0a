#!/bin/bash
# register / spill summary of one HIP source (compile-only): tools/regs.sh <file.hip> [extra flags]
f=$1; shift
cd $(dirname $(readlink -f $0))/../rl-k8s-scheduler_amd/csrc
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function -munsafe-fp-atomics "$@" -c $f -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys,re
name=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: name=m.group(1)[:60]
    m=re.search(r'VGPRs: (\d+)',l)
    if m: v=m.group(1)
    m=re.search(r'VGPRs Spill: (\d+)',l)
    if m: print(f'{name:62s} vgpr={v:>4s} spill={m.group(1)}')
    if 'error' in l: print(l.strip())
"
rm -f /tmp/regs_$$.o
