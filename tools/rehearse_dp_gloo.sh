#!/bin/bash
# 2-rank rehearsal of the data-parallel bench on ONE GPU (gloo; RCCL will not put two ranks on
# one device): the table exchanges (the bench's default 'best' = column at C3's width; the library's
# auto = gather) at C3 (in-batch loss, candidate-owner gradients) and the C5
# multiple-negatives workload.  Usage: bash tools/rehearse_dp_gloo.sh
set -o pipefail
run() {
  local tag=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --timing-steps 2 --dist-backend gloo \
    --no-cpu-baseline "$@" > gpurun_out/g2_$tag.log 2>&1 || exit $?
}
run best
run auto --table-sync auto
run column --table-sync column
run gather --table-sync gather
run shard --table-sync shard
run owner --table-sync owner
run c5 --config c5
