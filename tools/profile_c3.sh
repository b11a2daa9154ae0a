#!/bin/bash
# rocprofv3 evidence for the c3 node-level step kernel (run on the GPU box from the repo root):
# kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix / stalls)
# over tools/prof_step.py --c3 K.  Outputs under gpurun_out/prof_c3/.
set -e
R=$(pwd); O=$R/gpurun_out/prof_c3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c3 -- python3 $R/tools/prof_step.py --c3 100 > $O/trace.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python3 $R/tools/prof_step.py --c3 20 > $O/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python3 $R/tools/prof_step.py --c3 20 > $O/write.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM --output-format csv -d $O/pmc_sq1 -o p -- python3 $R/tools/prof_step.py --c3 20 > $O/sq1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $O/pmc_sq2 -o p -- python3 $R/tools/prof_step.py --c3 20 > $O/sq2.log 2>&1
python3 $R/tools/pmc_summary.py $O/summary.json $O/trace/c3_kernel_stats.csv \
  $O/pmc_fetch/p_counter_collection.csv $O/pmc_write/p_counter_collection.csv \
  $O/pmc_sq1/p_counter_collection.csv $O/pmc_sq2/p_counter_collection.csv > $O/summary.txt
cat $O/summary.txt
