#!/bin/bash
# Round-5 session C: C3 twiddle-load pricing.  kbench base / notw (twiddle pairs synthesised in
# registers, no loads; wrong results) / twlds (pairs 0..511 of both tables staged in LDS once per
# workgroup; exact), interleaved, two rounds, board power per run (tools/power_trace.sh).
set -o pipefail
OUT=gpurun_out/r5c; mkdir -p $OUT
export TMPDIR=/tmp
K=tools/kbench/bin
for i in 1 2; do
  for v in base notw twlds; do
    tools/power_trace.sh $OUT/tw$i $v $K/kbench_$v 4096 2013265921 65536 5000 || exit 1
    cat $OUT/tw$i/$v.out
  done
done 2>&1 | tee $OUT/tw.txt
echo done
