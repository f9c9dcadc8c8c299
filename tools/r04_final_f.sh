#!/bin/bash
# round-4 end: the other configurations on the final kernels (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04final
for cp in "c3 32" "c2 64" "c2 32" "c3z 64" "c3z 32"; do
  set -- $cp
  timeout -k 10 400 python3 bench.py --config $1 --precision $2 --steps 3 --warmup 1 --cpu-baseline none > gpurun_out/r04final/bench_$1_f$2.json 2> gpurun_out/r04final/bench_$1_f$2.err || { echo "$1 f$2 failed"; tail -5 gpurun_out/r04final/bench_$1_f$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04final/bench_$1_f$2.json')); r=d['roofline']
print('$1 f$2', d['ms_per_step'], r['kernel'], r['frac'], {k:(round(v['launch_ms'],1), v.get('frac')) for k,v in r['classes'].items()}, d['parity']['max_rel_err'])"
done
echo all-ok
