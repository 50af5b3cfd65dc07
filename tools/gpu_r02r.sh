#!/bin/bash
# AdamW scalars formed one step ahead (TT_ADAM_AHEAD): parity tests, A/B, timeline.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02r
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fusion.py tests/test_gpu_dp.py -k "adam or graph or side_stream or ahead or fusion or fused or bag_scaling or dp" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02r/test.log 2>&1 &&
tools/ab_bench.sh r02r_ab 3 "front:TT_ADAM_AHEAD=0" "ahead:TT_ADAM_AHEAD=1" "ahead_pre:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1" &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02r/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02r/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02r/kt/run_kernel_trace.csv > gpurun_out/r02r/timeline.txt
