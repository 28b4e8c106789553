#!/bin/bash
# Multi-pass kbench A/B at n = 8192 / 16384 / 32768 (u32, 31-bit q) and n = 16384 (62-bit q)
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for cfg in "8192 2013265921 8192" "16384 2013265921 4096" "32768 2013265921 2048" "16384 4611686018425815041 2048"; do
  VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh $cfg 100 >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
sort $OUT/ab.log | awk '{print $1, $2, $3, $5, $NF}'
