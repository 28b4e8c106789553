#!/bin/bash
# Round-5 session F: what the C3 kernel's vector-memory instruction count costs at the power cap:
# kbench base against a and b by 16-byte loads (x4l), c by 16-byte stores (x4s) and both (x4ls),
# the same bytes in a quarter of the instructions, registers unpermuted (wrong results); two
# interleaved rounds, board power per run.
set -o pipefail
OUT=gpurun_out/r5f; mkdir -p $OUT
export TMPDIR=/tmp
K=tools/kbench/bin
for i in 1 2; do
  for v in base x4l x4s x4ls; do
    tools/power_trace.sh $OUT/x4$i $v $K/kbench_$v 4096 2013265921 65536 5000 || exit 1
    cat $OUT/x4$i/$v.out
  done
done 2>&1 | tee $OUT/x4.txt
echo done
