#!/bin/bash
# Round-2 state at HEAD with the fused tail and pinned AdamW fmas: full GPU suite, smoke, default bench, then the round profile (kernel trace + PMC).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ze_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02ze_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02ze_bench.log 2>&1 &&
tools/profile_round.sh r02ze_c3 &&
python3 tools/step_timeline.py gpurun_out/r02ze_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02ze_c3/timeline.txt 2>&1
