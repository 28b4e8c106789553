#!/bin/bash
# Round-5 session E: C5 (square split) with the base multiplication's 128-bit sums from 31-bit limb
# products (NTTMUL_A64_LIMB=1: row pass 5,182 -> 4,783 VALU per thread, the same 1,100
# v_mad_u64_u32) against the default, three interleaved rounds, board power per run.
set -o pipefail
OUT=gpurun_out/r5e; mkdir -p $OUT
export TMPDIR=/tmp
K=tools/kbench/bin; Q=4611686018425815041
for i in 1 2 3; do
  for v in c5base c5limb; do
    tools/power_trace.sh $OUT/limb$i $v $K/kbench_$v 65536 $Q 1024 3000 || exit 1
    cat $OUT/limb$i/$v.out
  done
done 2>&1 | tee $OUT/limb.txt
echo done
