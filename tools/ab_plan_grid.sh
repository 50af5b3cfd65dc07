#!/bin/bash
# A/B of the plan grid cap: C3 bench step time, interleaved
for r in 1 2; do
  for g in 0 128 64 32; do
    echo "grid=$g run=$r $(TT_PLAN_GRID=$g timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --timing-steps 0 --no-helpers 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
