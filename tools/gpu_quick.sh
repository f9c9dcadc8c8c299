#!/bin/bash
# GPU tests + C3/C2 bench (no CPU baseline) — the inner loop of kernel work.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/tq.log 2>&1 || { echo "TESTS FAILED"; grep -E "^E |FAILED|Error" gpurun_out/tq.log | head -30; exit 1; }
tail -1 gpurun_out/tq.log
for cfg in ${CFGS:-c3 c2}; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bq_$cfg.json 2> gpurun_out/bq_$cfg.err || { echo "bench $cfg failed"; tail -5 gpurun_out/bq_$cfg.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bq_$cfg.json')); r=d['roofline']
print('$cfg', d['ms_per_step'], 'ms/epoch', d['value'], {k:(v['launch_ms'],v['tflops'],v['gbs']) for k,v in r['classes'].items()})"
done
