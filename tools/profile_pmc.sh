#!/bin/bash
# PMC passes for the bench's dominant kernel (run on the GPU box from the repo root).
# One counter group per rocprofv3 invocation, kernel-trace only (no sys/runtime trace with --pmc).
# Usage: tools/profile_pmc.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---no-cpu-baseline --steps 3 --warmup 1}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -T --kernel-include-regex 'k_rows|k_cols' \
    -d "$OUT/$name" -o "$name" --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
echo "pmc passes done: $OUT"
