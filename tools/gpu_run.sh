#!/bin/bash
# Generic GPU step: selected pytest targets (GPU marker) then the default bench.
# Usage: tools/gpu_run.sh TAG "pytest targets" [bench args...]
cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; TESTS=${2:-}; shift 2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1 || exit $?
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.log 2>&1
