#!/bin/bash
# A/B of the fused table-update reduce variants (TT_BAG_REDUCE) on the microbench, then FETCH_SIZE
# and TCC hit/miss per variant (separate rocprofv3 --pmc passes, kernel trace only).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abbag; mkdir -p $O
for v in ${VARIANTS:-rows rowsnt rows2 sliced slicednt rowsu8}; do
  TT_BAG_REDUCE=$v timeout -k 10 120 python tools/mb_bag_bwd.py >> $O/mb.log 2>&1
done
for v in ${PMC_VARIANTS:-rows sliced slicednt}; do
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | tr ' ' '_')
    TT_BAG_REDUCE=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/$v/$tag -o run -- python3 tools/mb_bag_bwd.py --iters 3 > $O/$v.$tag.log 2>&1
  done
done
