#!/bin/bash
# Deferred loss mean, high-priority wgrad side stream, bag prescale: parity tests, A/B, a timeline.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02n
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02n/test.log 2>&1 &&
tools/ab_bench.sh r02n_ab 3 "base:TT_BAG_PRESCALE=0 TT_DEFER_MEAN=0" "mean:TT_BAG_PRESCALE=0" "mean_prio:TT_BAG_PRESCALE=0 TT_SIDE_PRIO=wgrad" "pre_prio:TT_BAG_PRESCALE=1 TT_SIDE_PRIO=wgrad" &&
export TT_BAG_PRESCALE=1 TT_SIDE_PRIO=wgrad &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02n/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02n/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02n/kt/run_kernel_trace.csv > gpurun_out/r02n/timeline.txt
