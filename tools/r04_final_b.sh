#!/bin/bash
# round-4 end: PMC passes + kernel-trace stats of one C3 fp64 epoch (tools/pmc.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=c3 PREC=64 timeout -k 10 1100 bash tools/pmc.sh || exit 1
echo all-ok
