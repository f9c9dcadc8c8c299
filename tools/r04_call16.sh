#!/bin/bash
# round-4 GPU call 16: whitened x' pass with two gathered chunks in flight (QMFX_WB64_XD=2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_xd2.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_xd2.so" || exit 1
echo all-ok
