#!/bin/bash
# Fused combine + head L2 backward: parity tests; A/B with the bag prescale; timelines of each.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02m
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_kernels.py -k "fusion or fused or l2 or graph_step or side_stream or in_batch" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02m/test.log 2>&1 &&
tools/ab_bench.sh r02m_ab 3 "base:TT_BAG_PRESCALE=0 TT_FUSED_L2_BWD=0" "prescale:TT_BAG_PRESCALE=1 TT_FUSED_L2_BWD=0" "l2:TT_BAG_PRESCALE=0 TT_FUSED_L2_BWD=1" "both:TT_BAG_PRESCALE=1 TT_FUSED_L2_BWD=1" &&
for v in "base:TT_BAG_PRESCALE=0 TT_FUSED_L2_BWD=0" "both:TT_BAG_PRESCALE=1 TT_FUSED_L2_BWD=1" "prescale:TT_BAG_PRESCALE=1 TT_FUSED_L2_BWD=0"; do
  name=${v%%:*}; envs=${v#*:}
  export $envs
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02m/kt_$name -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02m/kt_$name.log 2>&1 || exit 1
  python3 tools/step_timeline.py gpurun_out/r02m/kt_$name/run_kernel_trace.csv > gpurun_out/r02m/timeline_$name.txt
done
