#!/bin/bash
# whitened buckets n = 65..128 at k = 256: tests, C3 A/B (old vs generalized kernel), C5 A/B (n > 64 direct vs whitened)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 700 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/wide.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/wide.test.log; exit 1; }
tail -1 gpurun_out/ab/wide.test.log
LIBS="var_old libqmfx" bash tools/s3_ab.sh || exit 1
CFG=c5 STEPS=2 bash tools/ab_env.sh "QMFX_WB_K256_NTN=4" "QMFX_WB_K256_NTN=8" "QMFX_WB_K256_NTN=4" "QMFX_WB_K256_NTN=8"
