#!/bin/bash
# Phase traces of the row kernels on C3-shaped halves (item half = direct rows, user half = whitened).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SIDE=1 timeout -k 10 300 python tools/trace_analyze.py > gpurun_out/trace_side1.txt 2>&1 || { echo "trace 1 failed"; tail gpurun_out/trace_side1.txt; exit 1; }
cat gpurun_out/trace_side1.txt
SIDE=0 timeout -k 10 300 python tools/trace_analyze.py > gpurun_out/trace_side0.txt 2>&1 || { echo "trace 0 failed"; tail gpurun_out/trace_side0.txt; exit 1; }
cat gpurun_out/trace_side0.txt
