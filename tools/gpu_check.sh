#!/bin/bash
# One GPU session: the given pytest selection (-m gpu), then tools/bench_runs.sh specs.
# usage: TESTS="tests/test_heavy_gpu.py tests/test_dist_gpu.py" tools/gpu_check.sh c3:64 c3z:64:1:1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/check
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/check/pytest.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/check/pytest.log | tail -40
  if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; tail -60 gpurun_out/check/pytest.log; exit $rc; fi
fi
if [ $# -gt 0 ]; then
  TAG=${TAG:-check} tools/bench_runs.sh "$@"
fi
