#!/bin/bash
# Round-2 re-entry (session 4): full GPU suite, smoke and default bench at HEAD.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02i_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02i_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02i_bench.log 2>&1
