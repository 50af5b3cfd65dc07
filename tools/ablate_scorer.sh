#!/bin/bash
# Timing ablations of the bf16 scorer engine (results are wrong by construction; timing only).
# Each variant rebuilds the library with -D flags and times tools/mb_scorer.py's C3 case.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ablate; mkdir -p $OUT; : > $OUT/res.log
for V in "" "-DTT_ABLATE_SREAD" "-DTT_ABLATE_BARRIER -DTT_ABLATE_EXP -DTT_ABLATE_ACCREAD" \
         "-DTT_ABLATE_BARRIER -DTT_ABLATE_EXP -DTT_ABLATE_ACCREAD -DTT_ABLATE_SREAD"; do
  rm -rf twotower_amd/csrc/build/scorer.hip.o
  make -C twotower_amd/csrc -j8 EXTRA="$V" > $OUT/build.log 2>&1
  echo "== [$V]" >> $OUT/res.log
  timeout -k 10 120 python3 tools/mb_scorer.py 2>/dev/null | head -1 >> $OUT/res.log
done
rm -rf twotower_amd/csrc/build/scorer.hip.o && make -C twotower_amd/csrc -j8 > /dev/null 2>&1
