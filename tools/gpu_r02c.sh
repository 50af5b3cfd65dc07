#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/scorer_error_table.py --tests > gpurun_out/r02c_err_tests.log 2>&1
