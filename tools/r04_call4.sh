#!/bin/bash
# round-4 GPU call 4: the two-wave fp64 direct kernel (wals_direct2.hip): WALS/config/heavy/
# CLI tests, then C3 fp64 A/B against the one-wave kernel (QMFX_DIRECT2=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py tests/test_heavy_gpu.py tests/test_dist_gpu.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04f/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04f/tests.log; exit 1; }
tail -2 gpurun_out/r04f/tests.log
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 600 bash tools/ab_env.sh "QMFX_DIRECT2=1" "QMFX_DIRECT2=0" "QMFX_DIRECT2=1" || exit 1
CFG=c2 PREC=64 STEPS=5 timeout -k 10 300 bash tools/ab_env.sh "QMFX_DIRECT2=1" "QMFX_DIRECT2=0" || exit 1
echo all-ok
