#!/bin/bash
# round-4 end: the driver's default line, exactly as the driver runs it, with its wall time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04final
t0=$(date +%s)
timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04final/default.json 2> gpurun_out/r04final/default.err
rc=$?
t1=$(date +%s)
echo "rc=$rc wall_s=$((t1 - t0))" | tee gpurun_out/r04final/default.wall.txt
cat gpurun_out/r04final/default.json
exit $rc
