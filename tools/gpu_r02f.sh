#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "in_batch" -v --timeout 120 --timeout-method thread > gpurun_out/r02f_ib.log 2>&1
