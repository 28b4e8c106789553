#!/bin/bash
# 30-bit q A/B (Arith32H vs Arith32P), 3 interleaved runs each at n = 4096 and n = 1024
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 4096 1073479681 65536 300 > $OUT/ab_4096.log 2>&1 || { cat $OUT/ab_4096.log; exit 1; }
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 1024 1073479681 262144 300 > $OUT/ab_1024.log 2>&1 || { cat $OUT/ab_1024.log; exit 1; }
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 256 12289 1048576 300 > $OUT/ab_256.log 2>&1 || { cat $OUT/ab_256.log; exit 1; }
cat $OUT/ab_4096.log $OUT/ab_1024.log $OUT/ab_256.log | sort | awk '{print $1, $2, $6, $NF}'
