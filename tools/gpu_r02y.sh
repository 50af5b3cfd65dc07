#!/bin/bash
# mean_kernel with its loads in flight: loss tests, kernel trace.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02y
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fusion.py -k "loss or triplet or multi or in_batch or golden or graph" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02y/test.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02y/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02y/kt.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/r02y/kt/run_kernel_trace.csv > gpurun_out/r02y/timeline.txt
