#!/bin/bash
# Round profile at HEAD (kernel trace + FETCH/WRITE PMC passes) and one replayed step's timeline.
cd "$GRAFT_REPO_ROOT"
tools/profile_round.sh r02j_c3 &&
python3 tools/step_timeline.py gpurun_out/r02j_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02j_c3/timeline.txt 2>&1
