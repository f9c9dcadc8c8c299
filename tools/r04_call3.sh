#!/bin/bash
# round-4 GPU call 3: the 4-column-panel fp64 Cholesky (chol4.h) -- full GPU suite on the
# in-tree library, then C3 fp64 A/B against the 16-column chol_solve build (var_chol16) and
# the phase traces of both halves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04d/gputests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r04d/gputests.log; exit 1; }
tail -2 gpurun_out/r04d/gputests.log
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 600 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_chol16.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" || exit 1
for side in 0 1; do
  echo "== trace side $side (chol4)"
  PREC=64 SIDE=$side timeout -k 10 300 python3 tools/trace_analyze.py 2>&1 | tail -n 8 || exit 1
done
echo all-ok
