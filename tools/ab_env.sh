#!/bin/bash
# Same-box A/B of environment settings on the C3 bench step (interleaved runs).
# Usage: tools/ab_env.sh RUNS 'VAR=a' 'VAR=b' ...   (an empty string: the default; BENCH_ARGS adds
# bench.py arguments, e.g. BENCH_ARGS="--config c5")
runs=$1; shift
for r in $(seq 1 "$runs"); do
  for e in "$@"; do
    ms=$(env $e timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --timing-steps 0 \
         --no-helpers $BENCH_ARGS 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "[$e] run=$r ms_per_step=$ms"
  done
done
