#!/bin/bash
# Round-6 bench lines, one bench process per configuration, each under its own time limit,
# stopping at the first failure.  Lines go to gpurun_out/lines/<name>.json (+ .err).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lines
mkdir -p "$OUT"
line() {  # name, limit, bench args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python3 -u bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { echo "$name FAILED"; tail -5 "$OUT/$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], 'ms/step', d['value'], d['unit'], r['kernel'], r['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'parity', (d.get('parity') or {}).get('pass'))" "$OUT/$name.json" "$name"
}
for spec in "$@"; do
  case $spec in
    c1) line bench_c1_f64 200 --config c1 ;;
    c2_32) line bench_c2_f32 300 --config c2 --precision 32 --steps 10 --warmup 2 ;;
    c2_64) line bench_c2_f64 300 --config c2 --precision 64 --steps 10 --warmup 2 --cpu-baseline none ;;
    c3_32) line bench_c3_f32 300 --config c3 --precision 32 --steps 5 --warmup 2 --cpu-baseline none ;;
    c3z_64) line bench_c3z_f64 300 --config c3z --precision 64 --steps 5 --warmup 2 --cpu-baseline none ;;
    c3z_32) line bench_c3z_f32 300 --config c3z --precision 32 --steps 5 --warmup 2 --cpu-baseline none ;;
    c4_64) line bench_c4_f64 400 --config c4 --precision 64 ;;
    c4_32) line bench_c4_f32 400 --config c4 --precision 32 ;;
    c5_64) line bench_c5_f64 300 --config c5 --precision 64 --steps 5 --warmup 2 --cpu-baseline sample ;;
    c5_32) line bench_c5_f32 300 --config c5 --precision 32 --steps 5 --warmup 2 --cpu-baseline none ;;
    c5z_64) line bench_c5z_f64 300 --config c5z --precision 64 --steps 5 --warmup 2 --cpu-baseline none ;;
    c5z_32) line bench_c5z_f32 300 --config c5z --precision 32 --steps 5 --warmup 2 --cpu-baseline none ;;
    *) echo "unknown spec $spec"; exit 2 ;;
  esac
done
