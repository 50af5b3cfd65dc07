cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pk
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in new base; do
  L=twotower_amd/libtwotower_amd.so; [ $v = base ] && L=tools/variants/lib_base.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk/$v/ks -o run -- python3 tools/mb_scorer_one.py 8192 16384 256 bf16 $L > gpurun_out/pk/$v.ks.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d gpurun_out/pk/$v/p1 -o run -- python3 tools/mb_scorer_one.py 8192 16384 256 bf16 $L > gpurun_out/pk/$v.p1.log 2>&1 || exit 1
  python3 tools/pmc_report.py gpurun_out/pk/$v > gpurun_out/pk/$v.txt 2>&1
done
