#!/bin/bash
# Round check on one GPU: the GPU test suite, smoke(), then the default bench (with the CPU
# baseline).  Usage: tools/gpu_suite_bench.sh TAG [pytest targets]
cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; TESTS=${2:-tests}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/suite.txt" 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> "$OUT/suite.txt" 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
