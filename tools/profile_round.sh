#!/bin/bash
# rocprofv3 evidence for the bench command (run on the GPU box from the repo root):
#   1. kernel trace + stats of `bench.py` itself (short run, no CPU baseline)
#   2. separate PMC passes over tools/prof_step.py: FETCH_SIZE, WRITE_SIZE, SQ instruction mix
# Outputs under gpurun_out/prof_<tag>/.  Every step has its own time limit; stop at the first failure.
set -e
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/bench_trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- \
  python3 $R/tools/prof_step.py --sgd 4 > $O/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- \
  python3 $R/tools/prof_step.py --sgd 4 > $O/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq1 -o p -- \
  python3 $R/tools/prof_step.py --sgd 4 > $O/pmc_sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $O/pmc_sq2 -o p -- \
  python3 $R/tools/prof_step.py --sgd 4 > $O/pmc_sq2.log 2>&1
python3 $R/tools/pmc_summary.py $O/summary.json $O/trace/bench_kernel_stats.csv \
  $O/pmc_fetch/p_counter_collection.csv $O/pmc_write/p_counter_collection.csv \
  $O/pmc_sq1/p_counter_collection.csv $O/pmc_sq2/p_counter_collection.csv > $O/summary.txt
cat $O/summary.txt
