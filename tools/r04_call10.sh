#!/bin/bash
# round-4 GPU call 10: fp64 panel columns broadcast through LDS instead of readlanes
# (chol.h QMFX_CHOL_LDSB): WALS/config/heavy tests, then C3 fp64 A/B against the readlane
# build (var_noldsb) and the round-start whitened kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04k
timeout -k 10 900 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py tests/test_heavy_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04k/tests.log; exit 1; }
tail -1 gpurun_out/r04k/tests.log
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_noldsb.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_wbhead.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_noldsb.so" || exit 1
SIDE=0 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04k/trace_side0.txt 2>&1 || { cat gpurun_out/r04k/trace_side0.txt; exit 1; }
SIDE=1 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04k/trace_side1.txt 2>&1 || { cat gpurun_out/r04k/trace_side1.txt; exit 1; }
cat gpurun_out/r04k/trace_side0.txt gpurun_out/r04k/trace_side1.txt
echo all-ok
