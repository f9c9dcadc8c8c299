#!/bin/bash
# A/B of the pre-fix direct kernel (QMFX_LIB=var_prev.so) vs the current library on C3 fp32, alternating
# in one box, then the C3 fp32 rocprofv3 kernel stats + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for i in 1 2; do
  for lib in var_prev libqmfx var_wbf32; do
    QMFX_LIB=$PWD/qmf_amd/_build/$lib.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline none --no-parity > gpurun_out/ab/$lib.$i.json 2> gpurun_out/ab/$lib.$i.err || { echo "bench failed $lib"; tail -5 gpurun_out/ab/$lib.$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab/$lib.$i.json')); r=d['roofline']
print('$lib $i', d['ms_per_step'], {k:round(v['launch_ms'],2) for k,v in r['classes'].items()})"
  done
done
[ -n "$NOPMC" ] || CFG=c3 PREC=32 bash tools/r02_pmc.sh
