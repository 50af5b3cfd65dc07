#!/bin/bash
# Round-2 re-entry (session 3): full GPU suite + default bench at HEAD.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02h_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02h_bench.log 2>&1
