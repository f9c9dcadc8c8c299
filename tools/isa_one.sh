#!/bin/bash
# ISA of selected row kernels without building the whole library: direct.h's (or
# SRC=woodbury.hip: woodbury.hip's) kernels with explicit instantiations only.  usage:
# SRC=woodbury.hip tools/isa_one.sh out.s "template __global__ void qmfx::wals_woodbury_kernel<float, 8, 4, false>(qmfx::SolveArgs<float>);" [-Dflags]
set -e
OUT=$1; INST=$2; shift 2
TU=$(mktemp /tmp/isa_one_XXXX.hip)
printf '#define QMFX_KERNELS_ONLY 1\n#include "%s/qmf_amd/csrc/%s"\n%s\n' "$(cd "$(dirname "$0")/.." && pwd)" "${SRC:-direct.h}" "$INST" > $TU
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize --cuda-device-only -S "$@" $TU -o $OUT -Rpass-analysis=kernel-resource-usage 2> ${OUT%.s}.res
rm -f $TU
