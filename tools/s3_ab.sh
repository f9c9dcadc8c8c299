#!/bin/bash
# same-box A/B of library variants on one bench config: LIBS="libqmfx var_x" [CFG=c3] [PREC=32] tools/s3_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for i in 1 2; do
  for lib in $LIBS; do
    QMFX_LIB=$PWD/qmf_amd/_build/$lib.so timeout -k 10 300 python bench.py --config ${CFG:-c3} --precision ${PREC:-32} --steps ${STEPS:-3} --warmup 1 --cpu-baseline none --no-parity > gpurun_out/ab/$lib.$i.json 2> gpurun_out/ab/$lib.$i.err || { echo "bench failed $lib"; tail -5 gpurun_out/ab/$lib.$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab/$lib.$i.json')); r=d['roofline']
print('$lib $i', d['ms_per_step'], {k:round(v['launch_ms'],2) for k,v in r.get('classes',{}).items()})"
  done
done
