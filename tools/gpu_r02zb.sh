#!/bin/bash
# Fused step tail (tt_adamw_multi_ex): its parity tests, the tests around the optimizer, a same-box
# A/B against the three launches it replaces, then a kernel trace + timeline of the default step.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_tail.py tests/test_gpu_kernels.py tests/test_gpu_fusion.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r02zb_gpu.log 2>&1 &&
tools/ab_bench.sh r02zb_ab 3 "tail3:TT_FUSED_TAIL=0" "fused:TT_FUSED_TAIL=1" &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02zb_kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02zb_kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02zb_kt/run_kernel_trace.csv > gpurun_out/r02zb_timeline.txt 2>&1
