#!/bin/bash
# round-4 end: the whole GPU test suite and smoke() on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04final/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r04final/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04final/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r04final/smoke.log; exit 1; }
tail -1 gpurun_out/r04final/smoke.log
echo all-ok
