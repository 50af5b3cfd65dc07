set -e
bash tools/profile_round.sh ${TAG:-r01f_c3} --steps 10 --warmup 3 --no-cpu-baseline
timeout -k 10 200 python bench.py > gpurun_out/${TAG:-r01f_c3}/bench.log 2>&1
