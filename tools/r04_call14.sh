#!/bin/bash
# round-4 GPU call 14: s_setprio around the whitened n×n factorization (timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NOPARITY=1 CFG=c3 PREC=64 STEPS=3 timeout -k 10 900 bash tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/libqmfx.so" "QMFX_LIB=qmf_amd/_build/var_prio1.so" "QMFX_LIB=qmf_amd/_build/var_prio2.so" "QMFX_LIB=qmf_amd/_build/var_priok.so" "QMFX_LIB=qmf_amd/_build/libqmfx.so" || exit 1
echo all-ok
