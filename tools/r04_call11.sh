#!/bin/bash
# round-4 GPU call 11: where the C5 big kernel spends its time (QMFX_ABLATE: 1 no Gram,
# 2 no panel factorisation, 4 no trailing update, 8 no backward solve), fp32 and fp64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04l
for p in 32 64; do
  PREC=$p MODES="0 1 2 4 8 14" timeout -k 10 500 python3 tools/ablate_half.py 10000000 1000000 500000000 256 > gpurun_out/r04l/ablate_c5_f$p.txt 2>&1 || { echo "ablate f$p failed"; tail -5 gpurun_out/r04l/ablate_c5_f$p.txt; exit 1; }
  echo "== f$p"; cat gpurun_out/r04l/ablate_c5_f$p.txt
done
echo all-ok
