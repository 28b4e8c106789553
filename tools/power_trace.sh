#!/bin/bash
# Board power and clocks while a workload runs (is the product kernel power-limited?).
# Usage (GPU box, repo root): tools/power_trace.sh <outdir> <label> <command...>
# Samples `amd-smi metric` (power, clocks, temperature) every ~0.3 s until the command exits;
# each sample is one JSON document in <outdir>/<label>.smi.jsonl, the command's stdout in
# <outdir>/<label>.out.  Read-only: no GPU setting is changed.
set -o pipefail
OUT=$1; LABEL=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 "$@" > "$OUT/$LABEL.out" 2> "$OUT/$LABEL.err" &
PID=$!
: > "$OUT/$LABEL.smi.jsonl"
while kill -0 $PID 2>/dev/null; do
  timeout -k 2 5 amd-smi metric -g 0 --json 2>/dev/null | tr -d '\n' >> "$OUT/$LABEL.smi.jsonl"
  echo >> "$OUT/$LABEL.smi.jsonl"
  sleep 0.3
done
wait $PID
rc=$?
echo "$LABEL rc=$rc samples=$(wc -l < "$OUT/$LABEL.smi.jsonl")"
exit $rc
