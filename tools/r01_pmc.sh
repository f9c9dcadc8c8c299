#!/bin/bash
# PMC passes over one C3 bench epoch (each counter group in its own rocprofv3 run,
# kernel-trace only), then phase ablations.  Outputs under gpurun_out/pmc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { echo "pmc $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "pmc $name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
run sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE
timeout -k 10 600 python tools/ablate_half.py > "$OUT/ablate.txt" 2>&1 || { echo "ablate failed"; tail "$OUT/ablate.txt"; exit 1; }
cat "$OUT/ablate.txt"
