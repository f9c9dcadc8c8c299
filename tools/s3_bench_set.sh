#!/bin/bash
# Round-2 session-3 bench set: every config's bench line (parity included; CPU baseline on C3 f32 and C4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02s3
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/r02s3/$name.json 2> gpurun_out/r02s3/$name.err || { echo "BENCH FAILED $name"; tail -20 gpurun_out/r02s3/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02s3/$name.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}
print('$name', d['ms_per_step'], d['value'], r.get('kernel'), r.get('frac'), (d.get('parity') or {}).get('max_rel_err'), cb.get('value'))"
}
run c3_f32 420 --steps 5 --warmup 1
run c3_f64 300 --precision 64 --steps 3 --warmup 1 --cpu-baseline none
run c2_f32 200 --config c2 --steps 5 --warmup 1 --cpu-baseline none
run c2_f64 200 --config c2 --precision 64 --steps 5 --warmup 1 --cpu-baseline none
run c4 300 --config c4 --steps 5 --warmup 1
run c5_f32 400 --config c5 --steps 2 --warmup 1 --cpu-baseline none
