cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab_noplan
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 --timing-steps 3 > gpurun_out/ab_noplan/plan_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/dbg/bench_noplan.py --no-cpu-baseline --steps 40 --timing-steps 3 > gpurun_out/ab_noplan/noplan_$i.log 2>&1 || exit $?
done
python3 tools/ab_summary.py gpurun_out/ab_noplan > gpurun_out/ab_noplan/summary.txt
