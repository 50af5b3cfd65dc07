#!/bin/bash
# Table reduce occupancy cap (TT_REDUCE_LDS) so the side-stream weight gradients are not starved,
# with the look-ahead AdamW scalars and the bag prescale: A/B + timelines.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02s
tools/ab_bench.sh r02s_ab 3 "front:TT_ADAM_AHEAD=0" "all:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1" "all_lds28:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1 TT_REDUCE_LDS=28672" "front_lds28:TT_REDUCE_LDS=28672" "all_lds24:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1 TT_REDUCE_LDS=24576" &&
for v in "all_lds28:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1 TT_REDUCE_LDS=28672" "all_lds24:TT_ADAM_AHEAD=1 TT_BAG_PRESCALE=1 TT_REDUCE_LDS=24576"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02s/kt_$name -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02s/kt_$name.log 2>&1 || exit 1
  python3 tools/step_timeline.py gpurun_out/r02s/kt_$name/run_kernel_trace.csv > gpurun_out/r02s/timeline_$name.txt
done
