#!/bin/bash
# Round profile of the bench step: a kernel-trace/stats pass and two PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), each its own rocprofv3 run with --kernel-trace only
# (never combined with sys/runtime/hip/hsa traces).  Usage: tools/profile_round.sh TAG [bench args]
set -e
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# --no-helpers: bench.py's scorer-attribution helpers (bench.py normalise_ms / l2_backward_ms) would
# otherwise land in the trace and be charged to the step
# --timing-steps 0: no stamped replay or eager timing pass after the timed steps (they would add
# a second capture's kernels and the stamp kernels to the trace)
ARGS="${*:---steps 10 --warmup 3 --no-cpu-baseline} --no-helpers --timing-steps 0 --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run -- \
  python3 bench.py $ARGS > "$OUT/ktrace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 bench.py $ARGS > "$OUT/write.log" 2>&1
python3 tools/summarize_profile.py "$OUT" "$TAG"
