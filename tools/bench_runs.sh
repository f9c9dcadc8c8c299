#!/bin/bash
# Runs bench.py once per "config:precision[:steps[:warmup]]" argument (no CPU baseline, parity
# on), each under its own time limit, stopping at the first failure.  Lines go to
# gpurun_out/runs/<tag>/<config>_<precision>.json (+ .err).
# usage: TAG=r03a tools/bench_runs.sh c3:64 c3z:32:1:1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/runs/${TAG:-run}"
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r cfg prec steps warm <<< "$spec"
  steps=${steps:-5}; warm=${warm:-2}
  echo "== $cfg fp$prec steps=$steps warmup=$warm"
  timeout -k 10 ${LIMIT:-400} python3 -u bench.py --config "$cfg" --precision "$prec" --steps "$steps" \
    --warmup "$warm" --cpu-baseline none ${EXTRA:-} > "$OUT/${cfg}_${prec}.json" 2> "$OUT/${cfg}_${prec}.err"
  rc=$?
  tail -3 "$OUT/${cfg}_${prec}.err"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], 'ms/epoch', d['value'], d['roofline']['kernel'], d['roofline']['frac'], {k: v['launch_ms'] for k, v in d['roofline']['classes'].items()}, d.get('parity', {}).get('max_rel_err'))" "$OUT/${cfg}_${prec}.json"
done
