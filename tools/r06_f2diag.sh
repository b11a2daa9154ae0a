#!/bin/bash
# round 6: the GPU suite on k_sf_dw2r as the default F2, then its time anatomy (timing-only F2R_DIAG
# builds: 1 no partial stores, 2 no MFMAs, 3 no production) beside k_sf_dw2 (RLKS_F2_IMAGE=1), same box
O=gpurun_out/r06_f2diag; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
line() {  # name config env...
  local n=$1 cf=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cf --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; return 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$n.txt') if l.startswith('{')][-1]
k=d['kernels']; print('$n', round(d['value']/1e6,3), 'ms/it', round(d['ms_per_step'],1), {n:round(v*1e3,1) for n,v in k['pipeline']['ms'].items()})"
}
line regs c4 X=1 && line image c4 RLKS_F2_IMAGE=1 && line d1_nostore c4 RLKS_LIB=$L/librlks_xp_d1.so && \
line d2_nomfma c4 RLKS_LIB=$L/librlks_xp_d2.so && line d3_noprod c4 RLKS_LIB=$L/librlks_xp_d3.so && line regs_b c4 X=1
