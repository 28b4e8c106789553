#!/bin/bash
# Round-5 session G: C3's unsigned Plantard product with its two v_mad_u64_u32 replaced by
# v_mul_lo_u32 + v_add3_u32 (th + 1) + v_mul_hi_u32 (phi2: -236 mads, +118 mul_lo / mul_hi /
# add3 per wave) and round 2's th + 1 form (phi1), against the base; two interleaved rounds,
# board power per run.
set -o pipefail
OUT=gpurun_out/r5g; mkdir -p $OUT
export TMPDIR=/tmp
K=tools/kbench/bin
for i in 1 2; do
  for v in base phi2 phi1; do
    tools/power_trace.sh $OUT/phi$i $v $K/kbench_$v 4096 2013265921 65536 5000 || exit 1
    cat $OUT/phi$i/$v.out
  done
done 2>&1 | tee $OUT/phi.txt
echo done
