#!/bin/bash
# A/B timing of one bench config under different environment settings (one bench process each).
# usage: CFG=c3 tools/ab_env.sh "ENV1=a ENV2=b" "ENV1=c" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for envs in "$@"; do
  env $envs timeout -k 10 300 python bench.py --config ${CFG:-c3} --precision ${PREC:-32} --no-cpu-baseline ${NOPARITY:+--no-parity} --steps ${STEPS:-2} > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed: $envs"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']
print('$envs |', d['ms_per_step'], 'ms/epoch |', {k:round(v['launch_ms'],2) for k,v in r['classes'].items()})"
done
