set -e
bash tools/profile_round.sh r01e_c3 --steps 10 --warmup 3 --no-cpu-baseline
timeout -k 10 200 python bench.py > gpurun_out/r01e_c3/bench.log 2>&1
