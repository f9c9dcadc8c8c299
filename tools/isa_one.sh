#!/bin/bash
# ISA of selected row kernels without building the whole library: wals.hip's (or
# SRC=woodbury: woodbury.hip's) kernels with explicit instantiations only.  usage: tools/isa_one.sh out.s "template __global__ void qmfx::wals_woodbury_kernel<float, 8, 4, false>(qmfx::SolveArgs<float>);" [-Dflags]
set -e
OUT=$1; INST=$2; shift 2
TU=$(mktemp /tmp/isa_one_XXXX.hip)
printf '#define QMFX_KERNELS_ONLY 1\n#include "%s/qmf_amd/csrc/%s.hip"\n%s\n' "$(cd "$(dirname "$0")/.." && pwd)" "${SRC:-wals}" "$INST" > $TU
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize --cuda-device-only -S "$@" $TU -o $OUT -Rpass-analysis=kernel-resource-usage 2> ${OUT%.s}.res
rm -f $TU
