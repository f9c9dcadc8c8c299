#!/bin/bash
# round-4 GPU call 2b: the k = 256 whole-row vs split check against the oracle, the fp64
# LDS-DMA Gram variants (tests, C3 A/B, trace), C4 at both precisions with the r04 PMC, C5z.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u -m pytest "tests/test_heavy_gpu.py::test_heavy_split_k256_matches_whole_row_kernel" -v --timeout 250 --timeout-method thread > gpurun_out/r04c/heavy256.log 2>&1
grep -E "PASS|FAIL|assert|Error" gpurun_out/r04c/heavy256.log | head -20
timeout -k 10 900 bash tools/ab_f64.sh var_glds7 var_glds5 > gpurun_out/r04c/ab_glds.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/r04c/ab_glds.log; exit 1; }
cat gpurun_out/r04c/ab_glds.log
for p in 64 32; do
  timeout -k 10 300 python3 bench.py --config c4 --precision $p --steps 5 --warmup 2 > gpurun_out/r04c/c4_f$p.json 2> gpurun_out/r04c/c4_f$p.err || { echo "c4 $p failed"; exit 1; }
done
echo c4-ok
for p in 64 32; do
  timeout -k 10 400 python3 bench.py --config c5z --precision $p --steps 2 --warmup 1 --cpu-baseline none > gpurun_out/r04c/c5z_f$p.json 2> gpurun_out/r04c/c5z_f$p.err || { echo "c5z $p failed"; tail -5 gpurun_out/r04c/c5z_f$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04c/c5z_f$p.json')); print('c5z', $p, d['ms_per_step'], d['parity']['max_rel_err'], {k:v['launch_ms'] for k,v in d['roofline']['classes'].items()})"
done
echo all-ok
