#!/bin/bash
# PMC HBM-traffic passes over one C3 epoch (one counter group per rocprofv3 run), then the
# other single-GPU bench lines (C2, C4 BPR, C5 k=256).  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { echo "pmc $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "pmc $name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
run sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py "$OUT" gpurun_out/pmc_c3_f32.json
for cfg in ${CFGS:-c2 c4 c5}; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  cat gpurun_out/bench_$cfg.json
done
