#!/bin/bash
# C5 fp32: whitened multi-wave (QMFX_WB_MW=1) vs streamed (QMFX_WB_MW=0) kernels, tests of the k=256 whitened path first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py -x -q -k "whitened or large_k or 256" --timeout 200 --timeout-method thread > gpurun_out/ab/c5.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/c5.test.log; exit 1; }
tail -1 gpurun_out/ab/c5.test.log
CFG=c5 STEPS=2 bash tools/ab_env.sh "QMFX_WB_MW=1" "QMFX_WB_MW=0" "QMFX_WB_MW=1" "QMFX_WB_MW=0"
