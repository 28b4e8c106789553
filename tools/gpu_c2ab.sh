#!/bin/bash
# n = 1024 kbench A/B (3 interleaved runs each, C2 batch and a long batch): tools/gpu_c2ab.sh <tag> "<variants>"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 1024 2013265921 4096 2000 > $OUT/ab_c2.log 2>&1 || { cat $OUT/ab_c2.log; exit 1; }
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 1024 2013265921 262144 200 > $OUT/ab_long.log 2>&1 || { cat $OUT/ab_long.log; exit 1; }
sort $OUT/ab_c2.log | awk '{print $1, $3, $6, $NF}'
sort $OUT/ab_long.log | awk '{print $1, $3, $6, $NF}'
