#!/bin/bash
# Bench lines for every single-GPU config (C3 default, C2, C4 BPR).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for cfg in c3 c2 c4; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  cat gpurun_out/bench_$cfg.json
done
