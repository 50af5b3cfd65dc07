#!/bin/bash
# fp32 scorer (C2) at H = 128 compiled for one wave per SIMD (no scratch spill) vs two (80 B/lane
# spill): scorer A/B at the C2 shape, the C2 parity tests on the variant, then the C2 step A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02zl
timeout -k 10 300 python -u tools/mb_variants.py --shape 4096 8192 128 --dtype fp32 \
  twotower_amd/libtwotower_amd.so tools/variants/lib_f32w1.so > gpurun_out/r02zl/mb.txt 2>&1 &&
TT_LIB=tools/variants/lib_f32w1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q \
  -k "c2" --timeout 300 --timeout-method thread > gpurun_out/r02zl/c2_tests.log 2>&1 &&
tools/ab_bench.sh r02zl/ab 3 "base:TT_PACK_INPUT=1" "f32w1:TT_LIB=tools/variants/lib_f32w1.so" -- --config c2
