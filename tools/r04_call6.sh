#!/bin/bash
# round-4 GPU call 6: is the two-wave fp64 direct Gram latency-bound?  Item-half phase trace
# with the gathers folded onto 1024 L2-resident rows (var_d2mask), C3 fp64 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04h
QMFX_LIB=qmf_amd/_build/var_d2mask.so SIDE=1 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04h/trace_d2mask.txt 2>&1 || { cat gpurun_out/r04h/trace_d2mask.txt; exit 1; }
cat gpurun_out/r04h/trace_d2mask.txt
NOPARITY=1 CFG=c3 PREC=64 STEPS=2 timeout -k 10 600 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/var_d2mask.so" "QMFX_LIB=qmf_amd/_build/var_gl2.so QMFX_DIRECT2=0" || exit 1
echo all-ok
