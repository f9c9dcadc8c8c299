#!/bin/bash
# PMC + kernel stats for C3 fp64 and C5 fp32 (the kernels changed this session)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=c3 PREC=64 bash tools/r02_pmc.sh && CFG=c5 PREC=32 bash tools/r02_pmc.sh
