#!/bin/bash
# Run GPU steps on the gpurun box, each under its own time limit; stop at the first crash/timeout.
# usage: tools/gpu_run.sh "<label>:<seconds>:<command>" ...
# A step whose exit code is 0 or 1 (pytest test failures) lets later steps run; any other code
# (abort, segfault, time limit) ends the script there.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$label] ($secs s) $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$label.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $label (rc=$rc)"; exit $rc; fi
done
exit 0
