#!/bin/bash
# rocprofv3 evidence for the c5 generic-width SGD step (tools/prof_wide.py): kernel trace + stats,
# then one SQ counter pass (separate run).  Outputs under gpurun_out/prof_<tag>/.
set -e
TAG=${1:-wide}
R=$(pwd)
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o wide -- \
  python3 $R/tools/prof_wide.py --reps 3 > $O/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o p -- \
  python3 $R/tools/prof_wide.py --reps 1 > $O/pmc_sq.log 2>&1
tail -3 $O/trace.log
