#!/bin/bash
# Same-box A/B of library builds on one bench config: one bench process per library
# (QMFX_LIB=<path>, "prod" = qmf_amd/_build/libqmfx.so), each under its own time limit.
# usage: CFG=c5 PREC=64 tools/ab_lib.sh prod qmf_amd/_build/var_x.so prod
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = prod ]; then unset QMFX_LIB; else export QMFX_LIB=$lib; fi
  timeout -k 10 ${LIMIT:-300} python3 -u bench.py --config ${CFG:-c5} --precision ${PREC:-64} \
    --steps ${STEPS:-2} --warmup ${WARM:-1} --cpu-baseline none ${NOPARITY:+--no-parity} --allow-variant \
    > gpurun_out/ab/$i.json 2> gpurun_out/ab/$i.err || { echo "bench failed: $lib"; tail -5 gpurun_out/ab/$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/$i.json')); r=d['roofline']
print('$lib |', d['ms_per_step'], 'ms/epoch |', {k:(v['per_side_launch_ms'], v['frac']) for k,v in r['classes'].items()}, d.get('parity',{}).get('max_rel_err'))"
done
