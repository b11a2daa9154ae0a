#!/bin/bash
set -e
R=$(pwd)
O=$R/gpurun_out/prof_split
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export RLKS_F1_SPLIT=1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o s -- python3 $R/tools/prof_step.py --sgd 16 > $O/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/sq -o p -- python3 $R/tools/prof_step.py --sgd 4 > $O/sq.log 2>&1
echo done
