#!/bin/bash
# 2-rank DP rehearsal (gloo, one GPU) with this session's defaults, both table exchanges and C5.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/rehearse_dp_gloo.sh && grep -h '"metric"' gpurun_out/g2_*.log | cut -c1-300 > gpurun_out/r02bb_dp.txt
