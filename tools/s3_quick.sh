#!/bin/bash
# quick GPU check: wals kernel tests + one C3 bench (no CPU baseline).  usage: TAG=x tools/s3_quick.sh [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s3
TAG=${TAG:-q}
timeout -k 10 600 python -u -m pytest tests/test_wals_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s3/$TAG.test.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/s3/$TAG.test.log; exit 1; }
tail -2 gpurun_out/s3/$TAG.test.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --cpu-baseline none "$@" > gpurun_out/s3/$TAG.json 2> gpurun_out/s3/$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/s3/$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/s3/$TAG.json')); r=d['roofline']
print(d['ms_per_step'], 'ms/epoch', d['parity']['max_rel_err'] if d.get('parity') else '', {k:round(v['launch_ms'],2) for k,v in r.get('classes',{}).items()})"
