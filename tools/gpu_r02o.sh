#!/bin/bash
# Weight gradients forked as soon as their operands exist (TT_WGRAD_EARLY), with / without the bag prescale.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "side_stream" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02o/test.log 2>&1 &&
TT_WGRAD_EARLY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fusion.py -k "side_stream or bag_scaling" -m gpu -x -q --timeout 200 --timeout-method thread >> gpurun_out/r02o/test.log 2>&1 &&
tools/ab_bench.sh r02o_ab 3 "base:TT_WGRAD_EARLY=0" "early:TT_WGRAD_EARLY=1" "early_pre:TT_WGRAD_EARLY=1 TT_BAG_PRESCALE=1" &&
export TT_WGRAD_EARLY=1 TT_BAG_PRESCALE=1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02o/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02o/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02o/kt/run_kernel_trace.csv > gpurun_out/r02o/timeline.txt
