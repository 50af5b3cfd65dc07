#!/bin/bash
# Launch-order variants: parity test, then a same-box A/B of the step time.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "launch_order or side_stream_wgrad or graph_step" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02k_test.log 2>&1 &&
tools/ab_bench.sh r02k_ab 3 "base:TT_EARLY_PREPARE=0" "prep_main:TT_EARLY_PREPARE=main" "prep_side:TT_EARLY_PREPARE=side" "defer:TT_PLAN_DEFER=1" "defer_side:TT_PLAN_DEFER=1 TT_EARLY_PREPARE=side"
