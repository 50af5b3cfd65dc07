#!/bin/bash
# Fused step tail (four threads per output for the slab sums) and the one-launch input pack:
# their tests, a same-box A/B of the three forms, then a kernel trace + timeline of the default.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_tail.py tests/test_gpu_kernels.py tests/test_gpu_fusion.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r02zc_gpu.log 2>&1 &&
tools/ab_bench.sh r02zc_ab 3 "base:TT_FUSED_TAIL=0 TT_PACK_INPUT=0" "tail:TT_FUSED_TAIL=1 TT_PACK_INPUT=0" \
  "tailpack:TT_FUSED_TAIL=1 TT_PACK_INPUT=1" &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02zc_kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02zc_kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02zc_kt/run_kernel_trace.csv > gpurun_out/r02zc_timeline.txt 2>&1
