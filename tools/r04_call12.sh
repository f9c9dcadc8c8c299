#!/bin/bash
# round-4 GPU call 12: fp64 k = 256 big kernel on the row-pair tile map (QMFX_BIG_PAIR64):
# k = 256 tests, then C5 fp64 A/B against the round-robin map (var_nopair).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04m
timeout -k 10 900 python -u -m pytest tests/test_wals_gpu.py tests/test_heavy_gpu.py -k "large_k or whitened or indefinite or k256 or chunked" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04m/tests.log; exit 1; }
tail -1 gpurun_out/r04m/tests.log
NOPARITY=1 CFG=c5 PREC=64 STEPS=2 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_nopair.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_nopair.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" || exit 1
echo all-ok
