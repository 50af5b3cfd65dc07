#!/bin/bash
# Sort plan forked before the gather (TT_PLAN_EARLY), now that the weight-gradient chain no longer starves.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02v
tools/ab_bench.sh r02v_ab 3 "base:TT_PLAN_EARLY=0" "early:TT_PLAN_EARLY=1" &&
TT_PLAN_EARLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02v/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02v/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02v/kt/run_kernel_trace.csv > gpurun_out/r02v/timeline.txt
