#!/bin/bash
# round-4 GPU call 5: phase traces of the C3 fp64 item half, two-wave direct kernel vs one wave.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
for v in 1 0; do
  QMFX_DIRECT2=$v SIDE=1 PREC=64 timeout -k 10 300 python -u tools/trace_analyze.py > gpurun_out/r04g/trace_direct2_$v.txt 2>&1 || { cat gpurun_out/r04g/trace_direct2_$v.txt; exit 1; }
  echo "== QMFX_DIRECT2=$v"; cat gpurun_out/r04g/trace_direct2_$v.txt
done
echo all-ok
