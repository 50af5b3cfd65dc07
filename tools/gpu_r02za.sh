#!/bin/bash
# Round-2 state at HEAD after the container restore: full GPU suite, smoke, default bench, then the round profile (kernel trace + PMC).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02za_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02za_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02za_bench.log 2>&1 &&
tools/profile_round.sh r02za_c3 &&
python3 tools/step_timeline.py gpurun_out/r02za_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02za_c3/timeline.txt 2>&1
