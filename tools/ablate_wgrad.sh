#!/bin/bash
# Timing ablations of the head weight-gradient kernel (results are wrong by construction).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ablate_wgrad; mkdir -p $OUT; : > $OUT/res.log
for V in "" "-DTT_WABL_NOMFMA" "-DTT_WABL_NOSTAGE" "-DTT_WABL_NOREAD" "-DTT_WABL_NOSTORE" \
         "-DTT_WABL_NOMFMA -DTT_WABL_NOSTAGE -DTT_WABL_NOREAD -DTT_WABL_NOSTORE"; do
  rm -rf twotower_amd/csrc/build/head.hip.o
  make -C twotower_amd/csrc -j8 EXTRA="$V" > $OUT/build.log 2>&1
  echo "== [$V]" >> $OUT/res.log
  timeout -k 10 120 python3 tools/mb_head.py 2>/dev/null | grep "head_wgrad" >> $OUT/res.log
done
rm -rf twotower_amd/csrc/build/head.hip.o && make -C twotower_amd/csrc -j8 > /dev/null 2>&1
