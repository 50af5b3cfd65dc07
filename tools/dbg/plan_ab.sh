cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/plan_ab
timeout -k 10 120 python tools/dbg/plan_ab.py gpurun_out/plan_ab/new.pt > gpurun_out/plan_ab/new.log 2>&1 &&
TT_LIB=tools/variants/lib_old.so timeout -k 10 120 python tools/dbg/plan_ab.py gpurun_out/plan_ab/old.pt > gpurun_out/plan_ab/old.log 2>&1 &&
python tools/dbg/plan_cmp.py gpurun_out/plan_ab/new.pt gpurun_out/plan_ab/old.pt > gpurun_out/plan_ab/cmp.txt 2>&1 &&
rm gpurun_out/plan_ab/*.pt &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "bag or fused or zipf or planned" -m gpu -x -q --timeout 300 > gpurun_out/plan_ab/tests.log 2>&1 &&
bash tools/ab_bench.sh ab_plan2 3 "new:TT_LIB=" "old:TT_LIB=tools/variants/lib_old.so"
