#!/bin/bash
# GPU check of the k <= 64 / fp64 paths: all WALS kernel tests, then C2 fp32 + fp64 and C3 fp64 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s3
TAG=${TAG:-c2}
timeout -k 10 700 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py tests/test_dist_gpu.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s3/$TAG.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/s3/$TAG.test.log; exit 1; }
tail -2 gpurun_out/s3/$TAG.test.log
for cfg in "c2 32" "c2 64" "c3 64"; do set -- $cfg
  timeout -k 10 400 python -u bench.py --config $1 --precision $2 --steps 3 --warmup 1 --cpu-baseline none > gpurun_out/s3/$TAG.$1_$2.json 2> gpurun_out/s3/$TAG.$1_$2.err || { echo BENCH FAILED $cfg; tail -20 gpurun_out/s3/$TAG.$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/s3/$TAG.$1_$2.json')); r=d['roofline']
print('$cfg', d['ms_per_step'], 'ms/epoch', d['parity']['max_rel_err'] if d.get('parity') else '', {k:round(v['launch_ms'],2) for k,v in r.get('classes',{}).items()})"
done
