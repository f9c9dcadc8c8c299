#!/bin/bash
# A/B timing of one bench config across library builds (QMFX_LIB), one bench process each.
# usage: CFG=c3 tools/ab_lib.sh qmf_amd/_build/libqmfx.so qmf_amd/_build/var_x.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  QMFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config ${CFG:-c3} --no-cpu-baseline --steps ${STEPS:-2} > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed: $lib"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 tools/ab_print.py gpurun_out/ab.json "$lib"
done
