#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that fails its tests (exit 1) lets
# the next one run, anything else (a time limit, an abort, a fault: 124, 134, 137, 139, ...) ends
# the call there.  Usage: tools/gpu_steps.sh SECONDS 'cmd' [SECONDS 'cmd' ...]
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  t=$1; cmd=$2; shift 2
  echo "[step] $cmd (limit ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd"
  rc=$?
  echo "[step] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] stopping: rc $rc"
    exit $rc
  fi
done
