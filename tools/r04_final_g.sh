#!/bin/bash
# round-4 end: C5 fp64 PMC passes + kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=c5 PREC=64 timeout -k 10 1000 bash tools/pmc.sh || exit 1
echo all-ok
