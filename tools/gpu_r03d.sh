cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 200 python -u tools/dbg/head_path_diag.py > $O/head_diag.txt 2>&1 || exit $?
TT_BAG_PRESCALE=0 timeout -k 10 200 python -u tools/dbg/head_path_diag.py > $O/head_diag_noprescale.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/mb_variants.py tools/variants/lib_base.so tools/variants/lib_unrollmap.so tools/variants/lib_umdefer.so tools/variants/lib_base.so tools/variants/lib_unrollmap.so tools/variants/lib_umdefer.so > $O/variants.txt 2>&1 || exit $?
NCCL_DEBUG=WARN timeout -k 10 300 python -X faulthandler -u bench.py --no-cpu-baseline --force-dist --table-sync shard --graph off --steps 4 --warmup 2 --timing-steps 1 > $O/force_shard_eager.json 2> $O/force_shard_eager.err || exit $?
NCCL_DEBUG=WARN timeout -k 10 300 python -X faulthandler -u bench.py --no-cpu-baseline --force-dist --table-sync gather --graph off --steps 4 --warmup 2 --timing-steps 1 > $O/force_gather_eager.json 2> $O/force_gather_eager.err || exit $?
