#!/bin/bash
# tools/profile_round.sh's three passes (kernel trace + stats, FETCH_SIZE, WRITE_SIZE; each its own
# rocprofv3 run with --kernel-trace only) over one tools/mb.py invocation instead of bench.py.
# Usage: tools/profile_mb.sh TAG mb-args...   (e.g. search_once)
set -e
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run -- \
  python3 tools/mb.py "$@" > "$OUT/ktrace.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 tools/mb.py "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 tools/mb.py "$@" > "$OUT/write.log" 2>&1
python3 tools/summarize_profile.py "$OUT" "$TAG"
