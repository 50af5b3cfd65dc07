#!/bin/bash
# Round profile at HEAD (fused combine + L2 backward default): kernel trace, FETCH/WRITE PMC passes, timeline.
cd "$GRAFT_REPO_ROOT"
tools/profile_round.sh r02p_c3 &&
python3 tools/step_timeline.py gpurun_out/r02p_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02p_c3/timeline.txt 2>&1
