#!/bin/bash
# round-2 first GPU pass: stored-P fix verification + scorer error table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3 4; do timeout -k 10 120 python -u tools/diag_inbatch_first.py >> gpurun_out/r02a_first.log 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "in_batch" -x -v --timeout 120 --timeout-method thread > gpurun_out/r02a_ib.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/scorer_error_table.py --big > gpurun_out/r02a_err.log 2>&1 || exit 1
