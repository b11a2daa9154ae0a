#!/bin/bash
# SQ anatomy (durations, MFMA busy, wave-cycle split, LDS activity / bank conflicts) of any profiling
# driver: pmc_any.sh <tag> <script relative to the repo> <args...>; summary via tools/pmc_anatomy.py <dir> <kernel substrings>
set -e
T=$1; shift
R=$(pwd)
S=$R/$1; shift  # the driver script, relative to the repo root
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $S "$@" > $O/trace.log 2>&1 || { echo trace failed; tail -5 $O/trace.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $O/a -o p -- python3 $S "$@" > $O/a.log 2>&1 || { echo pass a failed; tail -5 $O/a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/b -o p -- python3 $S "$@" > $O/b.log 2>&1 || { echo pass b failed; tail -5 $O/b.log; exit 1; }
