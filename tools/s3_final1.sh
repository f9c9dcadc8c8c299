#!/bin/bash
# full GPU test suite + smoke, then C3 fp32 PMC/stats for the current bucket layout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/final/gputest.log; exit 1; }
tail -1 gpurun_out/final/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
CFG=c3 PREC=32 bash tools/r02_pmc.sh
