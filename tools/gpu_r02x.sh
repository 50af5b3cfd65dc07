#!/bin/bash
# C5 (V 1M, multiple negatives): new defaults vs the round's earlier launch structure; timeline of each.
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02x
tools/ab_bench.sh r02x_ab 2 "new:TT_WGRAD2=1" "old:TT_WGRAD2=0 TT_BAG_PRESCALE=0 TT_ADAM_AHEAD=0" "w2only:TT_BAG_PRESCALE=0 TT_ADAM_AHEAD=0" -- --config c5 &&
for v in "new:TT_WGRAD2=1" "old:TT_WGRAD2=0 TT_BAG_PRESCALE=0 TT_ADAM_AHEAD=0"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02x/kt_$name -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 1 > gpurun_out/r02x/kt_$name.log 2>&1 || exit 1
  python3 tools/step_timeline.py gpurun_out/r02x/kt_$name/run_kernel_trace.csv > gpurun_out/r02x/timeline_$name.txt
done
