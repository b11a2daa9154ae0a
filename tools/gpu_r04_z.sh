#!/bin/bash
# HBM traffic of the c3 node step (work-list kernel, default build): kernel trace + FETCH_SIZE and
# WRITE_SIZE passes (MI355X_MICROARCH.md: separate passes, FETCH x 2 on gfx950), summarised
set -e
T=${1:-r04z}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $R/tools/node_step_time.py stationary > $O/trace.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c -o p -- python3 $R/tools/node_step_time.py stationary > $O/c.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/d -o p -- python3 $R/tools/node_step_time.py stationary > $O/d.log 2>&1
cd $R
python3 tools/pmc_anatomy.py $O k_node_step > /dev/null
rm -rf $O/trace $O/c $O/d
cat $O/summary.txt
