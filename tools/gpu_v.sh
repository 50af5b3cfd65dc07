cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_new.log 2>&1
