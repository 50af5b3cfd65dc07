cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pk &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "in_batch or inbatch or scorer" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ib.log 2>&1 &&
timeout -k 10 120 python -u tools/trace_scorer_bwd.py tools/variants/lib_trace.so > gpurun_out/traceb.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk/new/ks -o run -- python3 tools/mb_scorer_one.py 8192 16384 256 bf16 > gpurun_out/pk/new.ks.log 2>&1 &&
python3 tools/pmc_report.py gpurun_out/pk/new > gpurun_out/pk/new.txt 2>&1
