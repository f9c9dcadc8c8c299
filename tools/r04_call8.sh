#!/bin/bash
# round-4 GPU call 8: whitened fp64 kernel with the diagonal L blocks in the panel array
# (10.8 KB LDS per row at n <= 64) and one factorization call: whitened tests, then C3 fp64
# A/B against the round-start kernel (var_wbhead) and the 3/4-waves-per-SIMD builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py -k "whitened or large_k or indefinite or zero_and_negative" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04i/tests.log; exit 1; }
tail -2 gpurun_out/r04i/tests.log
for v in var_wb3 var_wb34 var_wbw34; do
  QMFX_LIB=qmf_amd/_build/$v.so timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py -k "whitened" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i/tests_$v.log 2>&1 || { echo "tests failed $v"; tail -40 gpurun_out/r04i/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04i/tests_$v.log)"
done
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_wbhead.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_wb3.so" "QMFX_LIB=qmf_amd/_build/var_wb34.so" "QMFX_LIB=qmf_amd/_build/var_wbw34.so" "QMFX_LIB=qmf_amd/_build/var_wbhead.so" || exit 1
echo all-ok
