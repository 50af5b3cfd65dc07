#!/bin/bash
# round-2 GPU pass b: in-batch tests (no -x) + scorer error table + C2 full-size tests
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/scorer_error_table.py --big > gpurun_out/r02b_err.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "in_batch" -v --timeout 120 --timeout-method thread > gpurun_out/r02b_ib.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 300 --timeout-method thread > gpurun_out/r02b_full.log 2>&1
