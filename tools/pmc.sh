#!/bin/bash
# PMC passes over one bench epoch of CFG at PREC (each counter group in its own rocprofv3
# run, kernel-trace only) plus a --stats kernel-trace run.  Outputs under
# gpurun_out/pmc_<CFG>_<PREC>/.  usage: CFG=c3 PREC=32 tools/pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${CFG:-c3}
PREC=${PREC:-32}
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_${CFG}_${PREC}"
mkdir -p "$OUT"
ARGS="--config $CFG --precision $PREC --steps 1 --warmup 1 --cpu-baseline none --no-parity"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" \
    -- python3 bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { echo "pmc $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "pmc $name ok"
}
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
  -- python3 bench.py $ARGS > "$OUT/stats.json" 2> "$OUT/stats.err" || { echo "stats failed"; exit 1; }
echo "stats ok"
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
run sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py "$OUT" "$OUT/pmc.json" && echo "summary ok"
