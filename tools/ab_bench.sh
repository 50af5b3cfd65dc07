#!/bin/bash
# Same-box A/B of bench variants: ROUNDS alternating runs of each variant.
# Usage: tools/ab_bench.sh TAG ROUNDS "name:ENV=v ENV2=v" "name2:..." [-- bench args]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1
TAG=$1; ROUNDS=$2; shift 2
VARS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for i in $(seq 1 $ROUNDS); do
  for v in "${VARS[@]}"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 --timing-steps 3 "$@" \
      > gpurun_out/$TAG/${name}_$i.log 2>&1 || exit $?
  done
done
python3 tools/ab_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt
