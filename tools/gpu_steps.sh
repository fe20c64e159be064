#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.  A step that
# fails with an ordinary test failure (exit 1) lets the next step run; a fault, abort, signal or
# time limit (any other non-zero status) ends the script there.
#   tools/gpu_steps.sh "<secs>|<name>|<cmd>" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after [$name] (rc=$rc)"; exit $rc; fi
done
exit 0
