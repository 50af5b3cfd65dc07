#!/bin/bash
# fp32 scorer at H = 128: forward at one wave per SIMD, backward at two (new default) vs both at
# two (lib_f32old): full GPU suite + smoke on the default, scorer A/B at C2, C2 step A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02zm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02zm/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r02zm/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u tools/mb_variants.py --shape 4096 8192 128 --dtype fp32 \
  tools/variants/lib_f32old.so twotower_amd/libtwotower_amd.so > gpurun_out/r02zm/mb.txt 2>&1 &&
tools/ab_bench.sh r02zm/ab 3 "old:TT_LIB=tools/variants/lib_f32old.so" "new:TT_PACK_INPUT=1" -- --config c2
