#!/bin/bash
# Deferred loss mean (formed by the backward combine's extra workgroup): its tests, the fusion
# tests, a same-box A/B against the mean's own launch, and a kernel trace + timeline.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_tail.py tests/test_gpu_fusion.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r02zf_gpu.log 2>&1 &&
tools/ab_bench.sh r02zf_ab 3 "mean:TT_DEFER_MEAN=0" "defer:TT_DEFER_MEAN=1" &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02zf_kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02zf_kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02zf_kt/run_kernel_trace.csv > gpurun_out/r02zf_timeline.txt 2>&1
