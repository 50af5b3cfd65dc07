#!/bin/bash
# Timing ablations of the split-bf16 head GEMM (results are wrong by construction; timing only).
# Each variant rebuilds the library with -D flags and times tools/mb_head.py's plain (epi 3) case.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ablate_head; mkdir -p $OUT; : > $OUT/res.log
M="-DTT_HABL_NOSTORE -DTT_HABL_NOSPLIT -DTT_HABL_NOALOAD -DTT_HABL_NOLDS -DTT_HABL_NOFILL"
for V in "$M" "$M -DTT_HABL_NOMFMA" "-DTT_HABL_NOSTORE -DTT_HABL_NOALOAD" "-DTT_HABL_NOSTORE -DTT_HABL_NOLDS"; do
  rm -rf twotower_amd/csrc/build/head.hip.o
  make -C twotower_amd/csrc -j8 EXTRA="$V" > $OUT/build.log 2>&1
  echo "== [$V]" >> $OUT/res.log
  timeout -k 10 120 python3 tools/mb_head.py 2>/dev/null | grep "epi 3" >> $OUT/res.log
done
rm -rf twotower_amd/csrc/build/head.hip.o && make -C twotower_amd/csrc -j8 > /dev/null 2>&1
