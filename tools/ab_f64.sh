#!/bin/bash
# fp64 direct-kernel variants: correctness (fp64 k = 96/128 direct rows against the oracle),
# then C3 fp64 A/B, then the item-half phase trace of each.  usage: tools/ab_f64.sh var1 var2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abf64
for v in "$@"; do
  QMFX_LIB=qmf_amd/_build/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    "tests/test_heavy_gpu.py::test_heavy_rows_match_oracle" "tests/test_wals_gpu.py::test_large_k_multiwave_rows" \
    "tests/test_configs_gpu.py" > gpurun_out/abf64/test_$v.log 2>&1 || { echo "TESTS FAILED $v"; tail -30 gpurun_out/abf64/test_$v.log; exit 1; }
  tail -n 1 gpurun_out/abf64/test_$v.log
done
args=()
for v in "$@"; do args+=("QMFX_LIB=qmf_amd/_build/$v.so"); done
CFG=c3 PREC=64 STEPS=3 tools/ab_env.sh "${args[@]}" || exit 1
for v in "$@"; do
  echo "== trace $v"
  QMFX_LIB=qmf_amd/_build/$v.so PREC=64 SIDE=1 timeout -k 10 300 python3 tools/trace_analyze.py 2>&1 | tail -n 6 || exit 1
done
