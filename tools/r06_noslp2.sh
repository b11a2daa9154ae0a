#!/bin/bash
# round 6: the library built with -fno-slp-vectorize as the default: GPU suite + smoke, then same-box
# c2 / c5 / c4 bench lines against the SLP build (librlks_xp_slp.so)
O=gpurun_out/r06_noslp2; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
L=$PWD/rl-k8s-scheduler_amd/rlks
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1))"
}
for c in c2 c5 c4; do
  line ${c}_noslp $c X=1 && line ${c}_slp $c RLKS_LIB=$L/librlks_xp_slp.so && line ${c}_noslp_b $c X=1 && line ${c}_slp_b $c RLKS_LIB=$L/librlks_xp_slp.so || exit 1
done
