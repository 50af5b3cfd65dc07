#!/bin/bash
# Kernel trace of the graph-replayed bench step only (no eager timing pass), for tools/step_timeline.py.
# Usage: tools/gpu_tl.sh TAG [bench args]
set -e
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --timing-steps 1 --no-cpu-baseline "$@" > gpurun_out/$TAG/bench.log 2>&1
f=$(ls gpurun_out/$TAG/kt/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/$TAG/kt/run_kernel_trace.csv)
python3 tools/step_timeline.py $f > gpurun_out/$TAG/timeline.txt
