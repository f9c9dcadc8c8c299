#!/bin/bash
# C3 users with 65..128 signals: direct (QMFX_WB_K128_NTN=4, default) vs whitened (8); tests with 8 first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
QMFX_WB_K128_NTN=8 timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/k128w.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/k128w.test.log; exit 1; }
tail -1 gpurun_out/ab/k128w.test.log
CFG=c3 STEPS=3 bash tools/ab_env.sh "QMFX_WB_K128_NTN=4" "QMFX_WB_K128_NTN=8" "QMFX_WB_K128_NTN=4" "QMFX_WB_K128_NTN=8"
