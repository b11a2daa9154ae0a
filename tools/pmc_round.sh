#!/bin/bash
# Round evidence for bench.py's roofline.traffic: the SGD-step PMC anatomy (tools/pmc_sgd.sh: c2 SGD
# steps of 65,536 rows, the c4 minibatch) and the c3 node step's FETCH / WRITE passes, each counter
# group in its own rocprofv3 run; writes gpurun_out/$1/pmc_traffic.json (copy to profiles/ to adopt).
set -e
T=${1:-pmc_round}
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p $O
bash tools/pmc_sgd.sh $T/sgd > $O/sgd.txt 2>&1 || { tail -20 $O/sgd.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/node_$C -o p -- python3 $R/tools/node_step_time.py stationary > $O/node_$C.log 2>&1 || { echo "node pass $C failed"; tail -5 $O/node_$C.log; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py $O/sgd/summary.json "profiles/$T: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/prof_step.py --sgd 16 (c2 SGD steps of 65,536 rows, the c4 minibatch); FETCH x 1024 x 2 + WRITE x 1024 per dispatch" $O/pmc_traffic.json > /dev/null
python3 tools/pmc_node_traffic.py $(ls $O/node_FETCH_SIZE/*counter_collection.csv) $(ls $O/node_WRITE_SIZE/*counter_collection.csv) "profiles/$T: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/node_step_time.py (65,536 envs x 8 x 256 nodes, stationary churn); FETCH x 1024 x 2 + WRITE x 1024 per dispatch" $O/pmc_traffic.json
cat $O/sgd/summary.txt
