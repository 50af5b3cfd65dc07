#!/bin/bash
# Plan-sort onesweep configurations measured on the whole step (the sort runs beside the head
# GEMMs and the scorer forward, whose CUs it takes): same-box A/B of variant libraries.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/ab_bench.sh r02zh_ab 3 "base:TT_PACK_INPUT=1" "p512x32:TT_LIB=tools/variants/lib_p512x32.so" \
  "p256x32:TT_LIB=tools/variants/lib_p256x32.so" "p1024x16:TT_LIB=tools/variants/lib_p1024x16.so"
