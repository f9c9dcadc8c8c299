#!/bin/bash
# C5 fp32 PMC/stats, then the bench set
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=c5 PREC=32 bash tools/r02_pmc.sh && bash tools/s3_bench_set.sh
