#!/bin/bash
# Onesweep configurations of the plan's radix sort, timed by tools/mb_plan.py (uniform and Zipf ids).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sweep_plan; mkdir -p $OUT; : > $OUT/res.log
for V in "-DTT_PLAN_BLOCK=1024 -DTT_PLAN_ITEMS=16 -DTT_PLAN_BITS=8" "-DTT_PLAN_BLOCK=256 -DTT_PLAN_ITEMS=16 -DTT_PLAN_BITS=8" \
         "-DTT_PLAN_BLOCK=512 -DTT_PLAN_ITEMS=8 -DTT_PLAN_BITS=8" "-DTT_PLAN_BLOCK=256 -DTT_PLAN_ITEMS=12 -DTT_PLAN_BITS=6" \
         "-DTT_PLAN_BLOCK=512 -DTT_PLAN_ITEMS=16 -DTT_PLAN_BITS=9" "-DTT_PLAN_BLOCK=256 -DTT_PLAN_ITEMS=8 -DTT_PLAN_BITS=9"; do
  rm -rf twotower_amd/csrc/build/bag.hip.o
  make -C twotower_amd/csrc -j16 EXTRA="$V" > $OUT/build.log 2>&1
  echo "== [$V]" >> $OUT/res.log
  timeout -k 10 120 python3 tools/mb_plan.py 2>/dev/null | grep "tt_bag_plan" >> $OUT/res.log
done
rm -rf twotower_amd/csrc/build/bag.hip.o && make -C twotower_amd/csrc -j16 > /dev/null 2>&1
