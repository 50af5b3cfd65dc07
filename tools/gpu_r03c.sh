cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u tools/mb_variants.py tools/variants/lib_base.so tools/variants/lib_unroll.so tools/variants/lib_unrollmap.so tools/variants/lib_base.so tools/variants/lib_unroll.so tools/variants/lib_unrollmap.so > $O/variants.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/dbg/step_grad_diag.py > $O/diag_c5.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/dbg/step_grad_diag.py 3000 128 24 96 1 in_batch > $O/diag_ib.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -m gpu -q --timeout 300 --timeout-method thread -k "reference_settings or dp" > $O/subset.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
for ts in shard gather; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --force-dist --table-sync $ts --steps 6 --warmup 3 --timing-steps 2 > $O/force_$ts.json 2> $O/force_$ts.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --force-dist --table-sync $ts --graph off --steps 6 --warmup 3 --timing-steps 2 > $O/force_${ts}_eager.json 2> $O/force_${ts}_eager.err || exit $?
done
