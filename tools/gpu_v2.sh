cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_new.log 2>&1
