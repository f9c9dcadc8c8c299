#!/bin/bash
# Round-4 timing experiments on the fp64 whitened class (C3 fp64): the in-tree library against
# variants that skip the n×n factorization (NOCHOL), serve the x' gather from L2 (XL2), skip
# the x' gather (NOX), or both (NOCHOL+NOX).  The variants compute wrong results; only their
# class times are read.  usage: tools/exp_r04_wb.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NOPARITY=1 CFG=c3 PREC=64 STEPS=2 tools/ab_env.sh "QMFX_LIB=qmf_amd/_build/libqmfx.so" \
  "QMFX_LIB=qmf_amd/_build/var_exp_nochol.so" "QMFX_LIB=qmf_amd/_build/var_exp_xl2.so" \
  "QMFX_LIB=qmf_amd/_build/var_exp_nox.so" "QMFX_LIB=qmf_amd/_build/var_exp_nocholnox.so"
