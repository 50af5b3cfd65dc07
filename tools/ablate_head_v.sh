#!/bin/bash
# Head GEMM timing ablations from prebuilt variant libraries (tools/build_variants.sh h*=...):
# tools/mb_head.py under TT_LIB for each.  Timing only (the ablated builds compute wrong results).
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ablate_head; mkdir -p $OUT; : > $OUT/res.log
for v in hbase hnosplit hnoaload hnostore hnolds hsplitload hmfma; do
  echo "== $v" >> $OUT/res.log
  TT_LIB=tools/variants/lib_$v.so timeout -k 10 120 python3 tools/mb_head.py >> $OUT/res.log 2>&1 || exit $?
done
