#!/bin/bash
# Same-box A/B of the single-process bf16 scorer's backward form (stored probabilities vs recompute)
# on the C3 step and the B x B pairs entry.  Usage: tools/ab_scorer_form.sh RUNS
for r in $(seq 1 "${1:-1}"); do
  for form in stored recompute; do
    TT_INBATCH_BWD=$form timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1 |
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=[x for x in d['kernels'] if x['op'].startswith('in-batch')][0]; b=d.get('scorer_bxb') or {}; print('$form', 'run=$r', 'c3_ms', d['ms_per_step'], 'c3_scorer_ms', k['mean_ms'], 'frac', k['frac'], 'bxb_ms', b.get('mean_ms'), 'bxb_frac', b.get('frac'), 'bxb_step_ms', b.get('step_ms'))"
  done
done
