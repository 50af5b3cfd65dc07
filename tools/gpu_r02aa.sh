#!/bin/bash
# l2_prep with 16-wave blocks: fusion parity tests, kernel trace + A/B against the previous library.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02aa
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_kernels.py -k "fusion or fused or prep or in_batch or graph" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02aa/test.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02aa/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02aa/kt.log 2>&1 &&
tools/ab_bench.sh r02aa_ab 3 "new:TT_LIB=" "old:TT_LIB=tools/variants/lib_prev.so"
