#!/bin/bash
# Round-2 end state: full GPU suite, smoke, the input-pack A/B (four loads per lane vs torch.cat),
# default bench, then the round profile (kernel trace + FETCH/WRITE PMC passes) and its timeline.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02zg_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02zg_smoke.log 2>&1 &&
tools/ab_bench.sh r02zg_ab 3 "cat:TT_PACK_INPUT=0" "pack:TT_PACK_INPUT=1" &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02zg_bench.log 2>&1 &&
tools/profile_round.sh r02zg_c3 &&
python3 tools/step_timeline.py gpurun_out/r02zg_c3/ktrace/run_kernel_trace.csv > gpurun_out/r02zg_c3/timeline.txt 2>&1
