#!/bin/bash
# Bag row scaling in the head's dx epilogue: parity tests, then a same-box A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "fusion or bag_scaling or graph_step or side_stream or planned or c3_step or bag_backward or head" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02l_test.log 2>&1 &&
tools/ab_bench.sh r02l_ab 3 "base:TT_BAG_PRESCALE=0" "prescale:TT_BAG_PRESCALE=1"
