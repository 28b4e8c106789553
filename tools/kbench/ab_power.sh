#!/bin/bash
# Interleaved kbench A/B with board power per run (GPU box, repo root):
#   tools/kbench/ab_power.sh <outdir> <rounds> "<kbench args>" <variant>...
# Each round runs every variant once (tools/kbench/bin/kbench_<variant> <kbench args>) under
# tools/power_trace.sh; prints each run's timing line (time, rate, output checksum) and writes the
# amd-smi samples to <outdir>/r<round>/<variant>.smi.jsonl (summarised by tools/summarize_power.py).
set -o pipefail
if [ "$1" = "--help" ] || [ $# -lt 4 ]; then
  sed -n 2,6p "$0"; exit 0
fi
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
K=$(dirname "$0")/bin
for i in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    "$(dirname "$0")/../power_trace.sh" "$OUT/r$i" "$v" $K/kbench_$v $ARGS || exit 1
    cat "$OUT/r$i/$v.out"
  done
done
