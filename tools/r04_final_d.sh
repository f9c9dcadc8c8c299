#!/bin/bash
# round-4 end: C5 (k = 256) benches at both precisions and the fp32 PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04final
for p in 32 64; do
  timeout -k 10 400 python3 bench.py --config c5 --precision $p --steps 3 --warmup 1 --cpu-baseline none > gpurun_out/r04final/bench_c5_f$p.json 2> gpurun_out/r04final/bench_c5_f$p.err || { echo "c5 f$p failed"; tail -5 gpurun_out/r04final/bench_c5_f$p.err; exit 1; }
  echo "c5 f$p ok"
done
CFG=c5 PREC=32 timeout -k 10 700 bash tools/pmc.sh || exit 1
echo all-ok
