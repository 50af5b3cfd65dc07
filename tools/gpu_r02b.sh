#!/bin/bash
# Round-2 profiles after the scorer rework: C3 and C5 kernel traces + FETCH/WRITE PMC passes,
# scorer SQ counters, and the default bench line.
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r02b_c3 --steps 10 --warmup 3 --no-cpu-baseline
bash tools/profile_round.sh r02b_c5 --config c5 --steps 10 --warmup 3 --no-cpu-baseline
bash tools/pmc_scorer.sh gpurun_out/r02b_scorer > /dev/null 2>&1
python3 tools/pmc_report.py gpurun_out/r02b_scorer > gpurun_out/r02b_scorer/report.txt 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r02b_c3/bench.log 2>&1
