#!/bin/bash
# Scorer PMC at HEAD (MFMA busy of both engines).
cd "$GRAFT_REPO_ROOT"
tools/pmc_scorer.sh gpurun_out/r02z_pmc bf16 &&
python3 tools/pmc_report.py gpurun_out/r02z_pmc gpurun_out/r02z_pmc/scorer_pmc.json > gpurun_out/r02z_pmc/report.txt
