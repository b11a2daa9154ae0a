#!/bin/bash
# (runs HERE, not on the GPU box: the gpurun client with a retry only while the pool has no free box)
# gpq.sh <log> <timeout> <cmd>: run gpurun, retrying only while no box/slot is free (nothing charged)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && grep -q "nothing was charged\|no free box\|backing off\|stopped responding while being prepared" $LOG; then
    echo "retry $i (rc=$rc)" >> $LOG.retries; sleep 150; continue
  fi
  break
done
echo "FINAL rc=$rc" >> $LOG
