#!/bin/bash
# Run GPU steps in order; stop at the first crash/abort/timeout (exit 124,134,137,139
# or >128), continue past ordinary failures (exit 1).  Usage:
#   tools/gpu_steps.sh "name1::seconds::cmd1" "name2::seconds::cmd2" ...
mkdir -p gpurun_out
rc_all=0
for spec in "$@"; do
  name="${spec%%::*}"; rest="${spec#*::}"; secs="${rest%%::*}"; cmd="${rest#*::}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  if [ $rc -ge 124 ]; then echo "=== stopping after crash/timeout in $name"; exit $rc; fi
done
exit $rc_all
