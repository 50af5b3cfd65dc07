cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -u tools/mb_variants.py tools/variants/lib_base.so tools/variants/lib_mapS.so tools/variants/lib_base.so tools/variants/lib_mapS.so > gpurun_out/r03a/variants.txt 2>&1 || exit $?
bash tools/gpu_suite_bench.sh r03a
