#!/bin/bash
# round-4 GPU call 9: whitened fp64 kernel keeping the first Zs chunks in registers for the
# x' pass (KEEP: n<=32 all 8, n<=48 4, n<=64 2): tests, C3 fp64 A/B, user-half trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py -k "whitened or large_k or indefinite or zero_and_negative" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04j/tests.log; exit 1; }
tail -1 gpurun_out/r04j/tests.log
QMFX_LIB=qmf_amd/_build/var_k35.so timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py -k "whitened" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j/tests_k35.log 2>&1 || { echo "tests failed k35"; tail -40 gpurun_out/r04j/tests_k35.log; exit 1; }
tail -1 gpurun_out/r04j/tests_k35.log
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_wbhead.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_k35.so" "QMFX_LIB=qmf_amd/_build/var_k0.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_wbhead.so" || exit 1
SIDE=0 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04j/trace_side0.txt 2>&1 || { cat gpurun_out/r04j/trace_side0.txt; exit 1; }
cat gpurun_out/r04j/trace_side0.txt
echo all-ok
