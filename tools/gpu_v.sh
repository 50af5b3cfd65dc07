cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "in_batch or inbatch or scorer" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ib.log 2>&1 &&
timeout -k 10 120 python -u tools/trace_scorer.py tools/variants/lib_trace.so > gpurun_out/trace2.log 2>&1 &&
timeout -k 10 300 python -u tools/mb_variants.py --iters 100 tools/variants/lib_base.so twotower_amd/libtwotower_amd.so tools/variants/lib_base.so twotower_amd/libtwotower_amd.so > gpurun_out/v3.log 2>&1
