#!/bin/bash
# round-4 GPU call 7: where the two-wave fp64 direct kernel's waves run (same SIMD or not).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04h
SIDE=1 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04h/trace_d2_simd.txt 2>&1 || { cat gpurun_out/r04h/trace_d2_simd.txt; exit 1; }
cat gpurun_out/r04h/trace_d2_simd.txt
echo all-ok
