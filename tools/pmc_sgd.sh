#!/bin/bash
# PMC anatomy of the SGD-step kernels (tools/prof_step.py: 16 c2 SGD steps of 65,536 rows, the c4
# PMC_CMD="tools/<script> <args>" / PMC_KEEP="<kernel substrings>" profile another driver (default: the SGD step)
# minibatch), one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: at most 8 SQ, 4 TCC
# (FETCH_SIZE 3, WRITE_SIZE 2), 2 GRBM per pass), plus a kernel-trace pass for durations.
# Summary (per dispatch averages, derived fractions) -> gpurun_out/$1/summary.txt / summary.json
R=$(pwd)
O=$R/gpurun_out/${1:-pmc_sgd}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o p -- python3 $R/${PMC_CMD:-tools/prof_step.py --sgd 16} > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }
}
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $R/${PMC_CMD:-tools/prof_step.py --sgd 16} > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
run a GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run c FETCH_SIZE
run d WRITE_SIZE
cd $R && python3 tools/pmc_anatomy.py $O $PMC_KEEP
