#!/bin/bash
# Run GPU steps in order, each under its own time limit; log to gpurun_out/<name>.log.
# A step that fails normally (exit 1: a failing test / assertion) does not stop the chain; a fault,
# abort, segfault or time-out (any other non-zero status) ends the script there.
#   scripts/gpu/steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)"; exit $rc
  fi
done
