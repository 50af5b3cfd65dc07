#!/bin/bash
# Kernel stats + two SQ counter passes (each its own rocprofv3 run, --kernel-trace only) over one
# tools/mb.py invocation.  Usage: tools/pmc_kernels.sh OUTDIR mb-args...   (e.g. scorer_once)
# Summarise with: python3 tools/pmc_report.py OUTDIR --match <kernel-name-substring>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/mb.py "$@" > $OUT/ks.log 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/mb.py "$@" > $OUT/p$i.log 2>&1
done
