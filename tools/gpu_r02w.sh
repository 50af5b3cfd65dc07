#!/bin/bash
# CW=2 stored-P backward (two candidate tiles per wave) with the fused combine + L2 backward; C2 and C5 benches at HEAD.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02w
TT_LIB=tools/variants/lib_cw2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_kernels.py -k "stored or fused" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02w/test.log 2>&1 &&
tools/ab_bench.sh r02w_ab 3 "cw1:TT_LIB=" "cw2:TT_LIB=tools/variants/lib_cw2.so" &&
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > gpurun_out/r02w/c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/r02w/c5.log 2>&1
