#!/bin/bash
# full GPU suite + round profile + default bench (stored-P backward default)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02d_pytest.log 2>&1 || exit 1
TAG=r02a_c3 bash tools/round_profile_and_bench.sh > gpurun_out/r02d_prof.log 2>&1 || exit 1
