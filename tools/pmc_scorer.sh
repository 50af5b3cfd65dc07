#!/bin/bash
# Scorer at B = 8192, H = 256: kernel stats + counter passes (each pass its own rocprofv3 run, --kernel-trace only).
# Usage: tools/pmc_scorer.sh OUTDIR [dtype] [M] [B] [H]  (defaults bf16 16384 8192 256: C3; M = 8192: the
# B x B pairs form; fp32 8192 4096 128: C2)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc_scorer}; DT=${2:-bf16}; M=${3:-16384}; B=${4:-8192}; H=${5:-256}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/mb.py scorer_once $B $M $H $DT > $OUT/ks.log 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/mb.py scorer_once $B $M $H $DT > $OUT/p$i.log 2>&1
done
