#!/bin/bash
# Timing experiments: build qmf_amd/_build/var_<name>.so = libqmfx with one source compiled
# under extra -D flags (csrc/wals.hip by default; SRC=woodbury tools/build_variant.sh ..., or
# SRCPATH=<path to a .hip> for an experimental copy, e.g. under tools/exp/).  The variant links a
# tag object, so qmfx_build_variant() returns its flags and bench.py refuses to report it as
# the product (unless --allow-variant, which marks the line).
# usage: tools/build_variant.sh name "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../qmf_amd"
B=_build
SRCFILE=${SRCPATH:-csrc/${SRC:-wals}.hip}
BASE=$(basename "$SRCFILE" .hip)
EXTRA=""
[ "$BASE" = "wals_direct_f64" ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -Icsrc $EXTRA $2 -c "$SRCFILE" -o $B/var_$1_src.o
printf 'extern "C" const char* qmfx_variant_flags_tag(void) { return "%s: %s %s"; }\n' "$1" "$(basename "$SRCFILE")" "$2" > $B/var_$1_tag.cpp
g++ -O2 -fPIC -c $B/var_$1_tag.cpp -o $B/var_$1_tag.o
OTHERS=$(ls $B/*.o | grep -v -e "/${BASE}.o\$" -e '/var_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $B/var_$1.so $B/var_$1_src.o $B/var_$1_tag.o $OTHERS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $B/var_$1_src.o $B/var_$1_tag.o $B/var_$1_tag.cpp
echo "built $B/var_$1.so"
