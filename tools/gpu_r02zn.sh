#!/bin/bash
# C2 (fp32 scorer) round profile at HEAD: kernel trace + FETCH/WRITE PMC passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/profile_round.sh r02zn_c2 --config c2 --steps 10 --warmup 3 --no-cpu-baseline &&
cp profiles/r02zn_c2_* gpurun_out/r02zn_c2/
