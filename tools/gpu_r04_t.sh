#!/bin/bash
# c3 node step ablations (prefetch / barrier) + one PMC pass over the default build
set -e
O=gpurun_out/${1:-r04t}; mkdir -p $O
L=$PWD/rl-k8s-scheduler_amd/rlks
for v in librlks librlks_xp_NOPF librlks_xp_FULLBAR librlks_xp_ec librlks librlks_xp_NOPF librlks_xp_FULLBAR; do
  echo "== $v" | tee -a $O/node_wl.txt
  RLKS_LIB=$L/$v.so timeout -k 10 120 python3 -u tools/node_step_time.py 2>&1 | grep -v amdgpu.ids | tee -a $O/node_wl.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc1 -o pmc -- python3 tools/node_step_time.py > $O/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/pmc2 -o pmc -- python3 tools/node_step_time.py > $O/pmc2.log 2>&1
