set -o pipefail
for ts in gather shard; do
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --timing-steps 2 --dist-backend gloo --table-sync $ts --no-cpu-baseline > gpurun_out/g2_$ts.log 2>&1 || exit $?
done
