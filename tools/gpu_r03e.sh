cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -q --timeout 300 --timeout-method thread -k "head or reference_settings or tower or row_ranges" > $O/subset.txt 2>&1
echo "subset rc=$?" >> $O/rc.txt
timeout -k 10 400 python -u tools/mb_variants.py tools/variants/lib_base.so tools/variants/lib_umdefer.so tools/variants/lib_udefer.so tools/variants/lib_base.so tools/variants/lib_umdefer.so tools/variants/lib_udefer.so tools/variants/lib_base.so tools/variants/lib_umdefer.so tools/variants/lib_udefer.so > $O/variants.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
NCCL_DEBUG=WARN timeout -k 10 300 python -X faulthandler -u bench.py --no-cpu-baseline --force-dist --table-sync gather --steps 4 --warmup 2 --timing-steps 1 > $O/force_gather_graph.json 2> $O/force_gather_graph.err || exit $?
