#!/bin/bash
# Both weight gradients in one side-stream launch, slab sums at the optimizer's join (TT_WGRAD2):
# parity tests, A/B with the look-ahead scalars and the bag prescale, timelines.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02t
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fusion.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py -k "head or wgrad or wgrad2 or side_stream or graph or adam or fusion or fused or bag_scaling or dp or c3_step" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02t/test.log 2>&1 &&
tools/ab_bench.sh r02t_ab 3 "old:TT_WGRAD2=0" "w2:TT_WGRAD2=1" "w2_all:TT_WGRAD2=1 TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1" "w2_ahead:TT_WGRAD2=1 TT_ADAM_AHEAD=1" &&
for v in "w2:TT_WGRAD2=1" "w2_all:TT_WGRAD2=1 TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02t/kt_$name -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02t/kt_$name.log 2>&1 || exit 1
  python3 tools/step_timeline.py gpurun_out/r02t/kt_$name/run_kernel_trace.csv > gpurun_out/r02t/timeline_$name.txt
done
