#!/bin/bash
# Timing experiments: build qmf_amd/_build/var_<name>.so = libqmfx with wals.hip compiled
# under extra -D flags (or another source: SRC=wals_big tools/build_variant.sh ...).
# usage: tools/build_variant.sh name "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../qmf_amd"
B=_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize $2 -c csrc/${SRC:-wals}.hip -o $B/var_$1_wals.o
OTHERS=$(ls $B/*.o | grep -v -e "/${SRC:-wals}.o\$" -e '/var_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $B/var_$1.so $B/var_$1_wals.o $OTHERS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $B/var_$1_wals.o
