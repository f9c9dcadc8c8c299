#!/bin/bash
# round-4 GPU call 13: whitened fp64 with one or two more Zs chunks kept in LDS for the x'
# pass (QMFX_WB64_KL*): whitened tests, then C3 fp64 A/B against var_nokl.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04n
timeout -k 10 900 python -u -m pytest tests/test_wals_gpu.py -k "whitened or indefinite or zero_and_negative or chunked or pieces" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04n/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04n/tests.log; exit 1; }
tail -1 gpurun_out/r04n/tests.log
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_nokl.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_nokl.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" || exit 1
echo all-ok
