#!/bin/bash
# Input pack, one unit per lane and one source per grid row: its tests, an A/B
# against torch.cat, the default bench and the round profile at HEAD.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_tail.py tests/test_gpu_fusion.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r02zj_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02zj_smoke.log 2>&1 &&
tools/ab_bench.sh r02zj_ab 3 "cat:TT_PACK_INPUT=0" "pack:TT_PACK_INPUT=1" &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02zj_bench.log 2>&1 &&
tools/profile_round.sh r02zj_c3 &&
python3 tools/step_timeline.py gpurun_out/r02zj_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02zj_c3/timeline.txt 2>&1
