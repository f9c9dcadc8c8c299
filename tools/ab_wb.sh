#!/bin/bash
# Kernel variants: parity (TESTS, default the whitened-bucket tests against the oracle), then
# a C3 A/B of each precision in PRECS against the in-tree library.
# usage: [TESTS="tests/x.py -k y"] tools/ab_wb.sh var1 var2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abwb
for v in "$@"; do
  QMFX_LIB=qmf_amd/_build/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_wals_gpu.py -k whitened} > gpurun_out/abwb/test_$v.log 2>&1 || { echo "TESTS FAILED $v"; tail -30 gpurun_out/abwb/test_$v.log; exit 1; }
  echo "$v: $(tail -n 1 gpurun_out/abwb/test_$v.log)"
done
args=("QMFX_LIB=qmf_amd/_build/libqmfx.so")
for v in "$@"; do args+=("QMFX_LIB=qmf_amd/_build/$v.so"); done
for p in ${PRECS:-64 32}; do
  echo "== fp$p"
  CFG=${CFG:-c3} PREC=$p STEPS=${STEPS:-3} tools/ab_env.sh "${args[@]}" || exit 1
done
