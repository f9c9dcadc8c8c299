#!/bin/bash
# tests of a library variant (QMFX_LIB), then a same-box A/B against the current library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
QMFX_LIB=$PWD/qmf_amd/_build/$VAR.so timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/$VAR.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/$VAR.test.log; exit 1; }
tail -1 gpurun_out/ab/$VAR.test.log
LIBS="libqmfx $VAR" bash tools/s3_ab.sh
