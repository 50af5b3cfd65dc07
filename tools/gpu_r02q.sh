#!/bin/bash
# Combine with all loads up front, l2_prep with 8 rows in flight: parity tests, kernel trace + timeline.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02q
timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "fusion or fused or in_batch or inbatch or scorer or c3 or stored" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02q/test.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02q/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02q/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02q/kt/run_kernel_trace.csv > gpurun_out/r02q/timeline.txt &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r02q/bench.log 2>&1
