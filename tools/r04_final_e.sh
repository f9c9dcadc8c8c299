#!/bin/bash
# round-4 end (after the last kernel change): C3 fp64 PMC + stats, then the driver's default
# line with its wall time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04final
CFG=c3 PREC=64 timeout -k 10 500 bash tools/pmc.sh || exit 1
t0=$(date +%s)
timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04final/default3.json 2> gpurun_out/r04final/default3.err
rc=$?
t1=$(date +%s)
echo "rc=$rc wall_s=$((t1 - t0))" | tee gpurun_out/r04final/default3.wall.txt
cat gpurun_out/r04final/default3.json
exit $rc
