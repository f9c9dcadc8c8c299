#!/bin/bash
# round-4 GPU call 15: s_setprio A/B for the whitened kernel (timing only), then the final
# C3 fp64 PMC + stats and the driver's default line with its wall time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/r04_call14.sh || exit 1
bash tools/r04_final_e.sh
