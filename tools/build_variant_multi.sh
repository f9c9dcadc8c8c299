#!/bin/bash
# Timing experiments: qmf_amd/_build/var_<name>.so = libqmfx with the listed sources rebuilt
# under extra -D flags (compiled in parallel; per-file Makefile flags kept).
# usage: tools/build_variant_multi.sh name "-DFOO=1" woodbury wals_direct_f64 ...
set -e
cd "$(dirname "$0")/../qmf_amd"
B=_build
name=$1; flags=$2; shift 2
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize"
pids=()
for src in "$@"; do
  extra=""
  [ "$src" = wals_direct_f64 ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc $F $extra $flags -Rpass-analysis=kernel-resource-usage -Icsrc -c $( [ -f csrc/$src.hip ] && echo csrc/$src.hip || echo ../tools/exp/$src.hip ) \
    -o $B/var_${name}_$src.o 2> $B/var_${name}_$src.ra &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
excl=""
for src in "$@"; do excl="$excl -e /$src.o\$"; done
OTHERS=$(ls $B/*.o | grep -v $excl -e '/var_')
# the tag object: qmfx_build_variant() reports this build's flags (bench.py refuses it as the product)
printf 'extern "C" const char* qmfx_variant_flags_tag(void) { return "%s: %s %s"; }\n' "$name" "$*" "$flags" > $B/var_${name}_tag.cpp
g++ -O2 -fPIC -c $B/var_${name}_tag.cpp -o $B/var_${name}_tag.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $B/var_$name.so $B/var_${name}_*.o $OTHERS \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $B/var_${name}_*.o $B/var_${name}_tag.cpp
