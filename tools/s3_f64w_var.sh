#!/bin/bash
# the fp64 wide-bucket patch built as qmf_amd/_build/var_f64w.so: WALS tests on it, then C3 fp64 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
L=$PWD/qmf_amd/_build/var_f64w.so
QMFX_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/f64w.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/f64w.test.log; exit 1; }
tail -1 gpurun_out/ab/f64w.test.log
CFG=c3 PREC=64 STEPS=2 bash tools/ab_env.sh "QMFX_LIB=$L QMFX_WB_F64_NTN=4" "QMFX_LIB=$L QMFX_WB_F64_NTN=5" "QMFX_LIB=$L QMFX_WB_F64_NTN=4" "QMFX_LIB=$L QMFX_WB_F64_NTN=5"
